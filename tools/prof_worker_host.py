#!/usr/bin/env python3
"""Host-side profile of the worker's sequential call (beam 5, VAD, 2 min clip, margin large-v3): cProfile over one
transcribe after a warm-up, top functions by cumulative and by own time.  Where the wall time goes between Python
and the library's C entry points (each C call includes its GPU wait).  Builder diagnostic."""
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vlog_amd.audio import speech_like, write_wav  # noqa: E402
from vlog_amd.transcribe import WhisperModel  # noqa: E402


def main():
    model = WhisperModel("synthetic:large-v3:0:margin", device="cpu", compute_type="int8")
    wav = os.path.join(tempfile.mkdtemp(), "c.wav")
    write_wav(wav, np.concatenate([speech_like(30.0, i) for i in range(4)]))

    def call():
        segs, info = model.transcribe(wav, language=None, task="transcribe", beam_size=5, vad_filter=True)
        return list(segs)

    call()
    t = time.perf_counter()
    call()
    print(f"wall {time.perf_counter() - t:.3f} s for 120 s of audio", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    call()
    pr.disable()
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(28)
        print(s.getvalue())


if __name__ == "__main__":
    main()
