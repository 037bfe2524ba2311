"""Work-balanced shards, measured on one GPU: the 2-GPU split of the variable-length workload
(large-v3, plant margin_var, 2 x 150 windows of the corpus), each rank's shard run in turn on the same GPU with the
bench's own pipeline (log-mel -> encoder -> row-set decode -> segments + WebVTT), for the two partitions of
vlog_amd/shard.py: by window count (partition_windows) and by expected tokens (partition_by_weight over the
frame-energy estimate).  The job's wall time is its slowest rank, so the ratio of the rank times is the figure.
Prints one JSON line.  Usage: shard_balance.py [world] [windows per rank] [steps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.shard import expected_tokens, partition_by_weight, partition_windows  # noqa: E402
from vlog_amd.tokenizer import Tokenizer  # noqa: E402
from vlog_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    Wn = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    dims = model_dims("large-v3")
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=0, plant="margin_var"), 0)
    tok = Tokenizer(dims, language="en")
    cache = {}
    est = []
    for r in range(world):                                # each rank's estimate of its natural range
        pcm, margin = bench.build_shard(r * Wn, Wn, cache, variable=True)
        db = eng.frame_energy_db(torch.from_numpy(pcm), 512)
        est.append(expected_tokens(db, 512, [margin + bench.CLIP * i for i in range(Wn)], [bench.CLIP] * Wn))
    est = np.concatenate(est)
    out = {"world": world, "windows": world * Wn, "steps": steps, "expected_tokens_total": float(est.sum())}
    n_total = world * Wn * bench.CLIP
    eng.reserve(2 * Wn, 2 * Wn)
    for name, parts in (("count", partition_windows(world * Wn, world)), ("tokens", partition_by_weight(est, world))):
        ranks = []
        for r, (g0, g1) in enumerate(parts):
            W = g1 - g0
            pcm, margin = bench.build_shard(g0, W, cache, variable=True)
            pipe = bench.Pipeline(eng, tok, dims, 0, 1, W, 1, torch.from_numpy(pcm).to(eng.device), margin, n_total,
                                  g0=g0, max_rows=0)
            pipe.step()                                   # warm-up (graphs, buffers)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                pipe.step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            ranks.append({"windows": [g0, g1], "s_per_step": round(dt, 4), "tokens": int(sum(pipe.last["tokens"])),
                          "expected": round(float(est[g0:g1].sum()), 1), "decoder_passes": pipe.last["steps"]})
            print(name, r, ranks[-1], file=sys.stderr, flush=True)
        t = [x["s_per_step"] for x in ranks]
        out[name] = {"ranks": ranks, "max_over_min": round(max(t) / min(t), 4),
                     "job_s_per_step": max(t), "rtfx_of_the_job": round(world * Wn * 30.0 / max(t), 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
