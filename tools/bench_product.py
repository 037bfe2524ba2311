#!/usr/bin/env python3
"""Builder-run throughput of the PRODUCT API on long-form audio (north_star: "synthetic long-form audio ...
concatenated to 1 h and 10 h"), not bench.py's step restatement:

  * `BatchedInferencePipeline.transcribe` through `WhisperModel(..., throughput=True).transcribe(pcm, ...)` — the
    call the unchanged worker makes with VLOG_AMD_THROUGHPUT=1 (reference worker/transcription.py:105-111) —
    timed from the call to the WebVTT string (log-mel, VAD off, encoder, batched greedy decode with timestamps,
    segment split, detokenise, generate_webvtt);
  * `ShardedTranscriber` (vlog_amd/shard.py, one spawned worker process per GPU; here N = 1 GPU) on the same PCM.

large-v3 with the margin-planted synthetic weights (decisive like a trained model, ~112 tokens per 30 s window),
the seeded speech-like corpus (clip i = speech_like(30 s, seed i)), PCM already in host memory (the worker's
WAV read is excluded, as is model load).  Prints one JSON line.
usage: python tools/bench_product.py [--hours 1 10] [--model large-v3] [--no-sharded]"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _clip(i):
    from vlog_amd.audio import speech_like
    return speech_like(30.0, i)


def corpus(hours: float) -> np.ndarray:
    n = int(round(hours * 120))
    with mp.get_context("spawn").Pool(min(16, os.cpu_count() or 4)) as pool:
        clips = pool.map(_clip, range(n), chunksize=8)
    return np.concatenate(clips).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hours", type=float, nargs="+", default=[1.0, 10.0])
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--no-sharded", action="store_true")
    args = ap.parse_args()
    spec = f"synthetic:{args.model}:0:margin"
    pcms = {h: corpus(h) for h in args.hours}
    out = {"model": spec, "mode": "greedy, timestamps, language en, vad_filter False", "n_gpus": 1, "runs": {}}
    sharded = None
    if not args.no_sharded:
        # the coordinator must not touch the GPU before spawning its workers
        from vlog_amd.shard import ShardedTranscriber
        sharded = ShardedTranscriber(spec, [0])
        for h, pcm in pcms.items():
            sharded.transcribe(pcm[: 16000 * 60], language="en", beam_size=1, without_timestamps=False)   # warm-up
            t = time.perf_counter()
            segs = sharded.transcribe(pcm, language="en", beam_size=1, temperature=0.0, without_timestamps=False)
            from vlog_amd.vtt import generate_webvtt
            vtt = generate_webvtt(segs)
            dt = time.perf_counter() - t
            out["runs"][f"sharded_{h:g}h"] = {"api": "ShardedTranscriber([0]).transcribe", "audio_s": len(pcm) / 16000,
                                              "wall_s": round(dt, 3), "rtfx": round(len(pcm) / 16000 / dt, 1),
                                              "segments": len(segs), "vtt_bytes": len(vtt)}
            print(json.dumps(out["runs"][f"sharded_{h:g}h"]), file=sys.stderr, flush=True)
        sharded.close()
    from vlog_amd.transcribe import WhisperModel
    from vlog_amd.vtt import generate_webvtt
    model = WhisperModel(spec, device="cpu", compute_type="int8", throughput=True)

    def call(pcm):
        t = time.perf_counter()
        segments, info = model.transcribe(pcm, language="en", task="transcribe", beam_size=1, temperature=0.0,
                                          vad_filter=False, without_timestamps=False)
        segs = [{"start": s.start, "end": s.end, "text": s.text} for s in segments]
        vtt = generate_webvtt(segs)
        return time.perf_counter() - t, segs, vtt

    call(pcms[args.hours[0]][: 16000 * 120])                                   # warm-up
    for h, pcm in pcms.items():
        dt, segs, vtt = call(pcm)
        out["runs"][f"batched_{h:g}h"] = {"api": "WhisperModel(throughput=True).transcribe -> BatchedInferencePipeline",
                                          "audio_s": len(pcm) / 16000, "wall_s": round(dt, 3),
                                          "rtfx": round(len(pcm) / 16000 / dt, 1), "segments": len(segs),
                                          "vtt_bytes": len(vtt)}
        print(json.dumps(out["runs"][f"batched_{h:g}h"]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
