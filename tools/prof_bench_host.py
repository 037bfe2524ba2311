#!/usr/bin/env python3
"""Host-side profile of one bench.py step (builder diagnostic): the bench's own Pipeline on large-v3 (150 windows),
one warm-up step, then cProfile over one step.  Usage: prof_bench_host.py [beam] [words 0|1] [variable 0|1]"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.tokenizer import Tokenizer  # noqa: E402
from vlog_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    beam = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    words = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    variable = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    W = 150
    dims = model_dims("large-v3")
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=0, plant="margin_var" if variable else "margin"), 0)
    if beam > 1:
        eng.set_option("cross_mode", 0)
    tok = Tokenizer(dims, language="en")
    pcm, margin = bench.build_shard(0, W, {}, variable=bool(variable))
    eng.reserve(W, W * beam)
    pipe = bench.Pipeline(eng, tok, dims, 0, 1, W, beam, torch.from_numpy(pcm).to(eng.device), margin, W * bench.CLIP,
                          words=bool(words), max_rows=0 if variable else -1)
    pipe.step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    pipe.step()
    torch.cuda.synchronize()
    print(f"step {time.perf_counter() - t:.3f} s; stages {pipe.stage}", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    pipe.step()
    torch.cuda.synchronize()
    pr.disable()
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
        print(s.getvalue())


if __name__ == "__main__":
    main()
