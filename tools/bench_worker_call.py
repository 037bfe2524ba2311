#!/usr/bin/env python3
"""Builder-run benchmark of the UNCHANGED worker's exact call (reference worker/transcription.py:81-85, 105-133):

    model = WhisperModel(WHISPER_MODEL, device="cpu", compute_type="int8")
    segments, info = model.transcribe(str(wav), language=None, task="transcribe", beam_size=5, vad_filter=True)
    for segment in segments: ...; text = " ".join(...); captions = generate_webvtt(...)

timed from the call to the VTT string, in the default sequential mode (faster-whisper seek loop) and in the
opt-in throughput mode (VLOG_AMD_THROUGHPUT=1 -> BatchedInferencePipeline).  Reports RTFx of each and the WER
of the throughput transcript against the sequential one on the same clip.  Synthetic large-v3 weights with the
margin-planted decoder program (decisive like a trained model: windows pass faster-whisper's thresholds at
temperature 0, so the default fallback ladder costs nothing extra); --random-weights: plain random init, whose
average log-probability (about -7) fails the -1.0 threshold on every window, so the fallback re-decodes every
window at five temperatures (best_of 5).  Prints one JSON line.
usage: python tools/bench_worker_call.py [--minutes-seq 5] [--minutes-tp 60] [--model large-v3]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from vlog_amd.audio import speech_like, write_wav  # noqa: E402
from vlog_amd.metrics import word_error_rate  # noqa: E402
from vlog_amd.transcribe import WhisperModel  # noqa: E402
from vlog_amd.vtt import generate_webvtt  # noqa: E402


def worker_call(model, wav, temperature=None):
    """The worker's TranscriptionWorker.transcribe + generate_webvtt (worker/transcription.py:92-133, 377).
    temperature=None keeps faster-whisper's default fallback ladder (the worker's call as written)."""
    t = time.perf_counter()
    kw = {} if temperature is None else {"temperature": temperature}
    segments, info = model.transcribe(str(wav), language=None, task="transcribe", beam_size=5, vad_filter=True, **kw)
    segs, parts = [], []
    for s in segments:
        segs.append({"start": s.start, "end": s.end, "text": s.text})
        parts.append(s.text.strip())
    vtt = generate_webvtt(segs)
    return time.perf_counter() - t, " ".join(parts), info, len(segs), len(vtt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--minutes-seq", type=float, default=5.0)
    ap.add_argument("--minutes-tp", type=float, default=60.0)
    ap.add_argument("--temperature", type=float, default=None,
                    help="fixed temperature (e.g. 0: no fallback ladder, the cost of the call on a model whose windows "
                         "pass faster-whisper's thresholds); default: the worker's call as written")
    ap.add_argument("--random-weights", action="store_true",
                    help="plain random-init weights (every window fails the log-prob threshold and is re-decoded at "
                         "five temperatures); default: the margin-planted model, whose windows pass like a trained one")
    ap.add_argument("--no-graph", action="store_true", help="decode steps launched eagerly (decode_graph=0)")
    args = ap.parse_args()
    spec = f"synthetic:{args.model}:0" + ("" if args.random_weights else ":margin")
    model = WhisperModel(spec, device="cpu", compute_type="int8", eot_after=110)
    if args.no_graph:
        model.engine.set_option("decode_graph", 0)
    tmp = tempfile.mkdtemp()

    def clip(minutes, name):
        n = int(round(minutes * 2))
        path = os.path.join(tmp, name)
        write_wav(path, np.concatenate([speech_like(30.0, i) for i in range(n)]))
        return path, n * 30.0

    short, short_s = clip(args.minutes_seq, "short.wav")
    long_, long_s = clip(args.minutes_tp, "long.wav")
    out = {"model": args.model, "weights": spec, "decode_graph": not args.no_graph, "call": "transcribe(str(wav), language=None, task='transcribe', beam_size=5, "
                                        "vad_filter=True) + generate_webvtt"}
    T = args.temperature
    if T is not None:
        out["temperature"] = T
    model.throughput = True
    worker_call(model, short, T)                                   # warm-up (allocations, kernels)
    model.throughput = False
    dt, text_seq, info, nseg, _ = worker_call(model, short, T)
    out["sequential"] = {"audio_s": short_s, "wall_s": round(dt, 3), "rtfx": round(short_s / dt, 2), "segments": nseg,
                         "duration_after_vad": round(info.duration_after_vad, 2)}
    model.throughput = True
    dt, text_tp, info, nseg, _ = worker_call(model, short, T)
    out["throughput_same_clip"] = {"audio_s": short_s, "wall_s": round(dt, 3), "rtfx": round(short_s / dt, 2),
                                   "segments": nseg}
    out["wer_throughput_vs_sequential"] = round(word_error_rate(text_seq, text_tp), 4)
    dt, _, info, nseg, _ = worker_call(model, long_, T)
    out["throughput"] = {"audio_s": long_s, "wall_s": round(dt, 3), "rtfx": round(long_s / dt, 2), "segments": nseg,
                         "duration_after_vad": round(info.duration_after_vad, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
