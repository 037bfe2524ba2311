#!/usr/bin/env python3
"""Per-kernel-class time of the worker's default call in sequential mode (beam 5, VAD, temperature ladder) on a
short clip, from the engine's event profiler (builder diagnostic).  Prints one JSON line."""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vlog_amd.audio import speech_like, write_wav  # noqa: E402
from vlog_amd.transcribe import WhisperModel  # noqa: E402


def main():
    # usage: prof_worker_seq.py [model] [opt=value,opt=value]  (engine options, e.g. decode_gemm.qkv=-1)
    model = WhisperModel(f"synthetic:{sys.argv[1] if len(sys.argv) > 1 else 'large-v3'}:0:margin", device="cpu",
                         compute_type="int8")
    opts = {}
    if len(sys.argv) > 2 and sys.argv[2]:
        for kv in sys.argv[2].split(","):
            k, v = kv.split("=")
            opts[k] = int(v)
            model.engine.set_option(k, int(v))
    wav = os.path.join(tempfile.mkdtemp(), "c.wav")
    write_wav(wav, np.concatenate([speech_like(30.0, i) for i in range(2)]))
    list(model.transcribe(wav, beam_size=5)[0])              # warm-up
    eng = model.engine
    eng.profile(True)
    t = time.perf_counter()
    segs = list(model.transcribe(wav, beam_size=5)[0])
    dt = time.perf_counter() - t
    eng.profile(False)
    prof = {k: {"launches": v["launches"], "ms": round(v["ms"], 3)} for k, v in eng.profile_read().items() if v["launches"]}
    print(json.dumps({"opts": opts, "wall_s": round(dt, 3), "audio_s": 60.0, "rtfx": round(60.0 / dt, 1), "segments": len(segs),
                      "gpu_ms_by_class": prof, "sum_gpu_ms": round(sum(v["ms"] for v in prof.values()), 1)}))


if __name__ == "__main__":
    main()
