#!/usr/bin/env python3
"""Probe (tools only): how much of the encoder can hide under the decoder on one MI355X.  Two engines with the
bench's large-v3 weights on two streams, driven from two threads (ctypes releases the GIL): engine A loops
the 150-window decode (generate), engine B loops the 150-window encoder.  Prints each alone and both at once,
as seconds per iteration and the fraction of the serial time the overlap saves."""
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from vlog_amd.audio import speech_like  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.tokenizer import Tokenizer  # noqa: E402
from vlog_amd.weights import synthetic_state_dict  # noqa: E402

W = int(os.environ.get("PROBE_WINDOWS", "150"))
ITERS = int(os.environ.get("PROBE_ITERS", "3"))

dims = model_dims("large-v3")
sd = synthetic_state_dict(dims, seed=0, eot_after=110)
ea = GpuEngine(dims, sd, 0)
eb = GpuEngine(dims, sd, 0)
del sd
pcm = torch.from_numpy(np.concatenate([speech_like(30.0, i) for i in range(W)])).cuda()
mel = ea.features(pcm)
enc = ea.encode(mel, [3000 * i for i in range(W)], [3000] * W)
ea.reserve(W, W)
ea.cross_kv(enc, 0)
tok = Tokenizer(dims, language="en")
prompt = list(tok.sot_sequence)
sup = list(tok.suppressed_tokens([-1]))
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def decode_loop(n, out):
    with torch.cuda.stream(sa):
        t = time.perf_counter()
        for _ in range(n):
            ea.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=448, check_every=8)
        torch.cuda.synchronize()
        out["decode"] = (time.perf_counter() - t) / n


def encode_loop(n, out):
    with torch.cuda.stream(sb):
        t = time.perf_counter()
        for _ in range(n):
            eb.encode(mel, [3000 * i for i in range(W)], [3000] * W)
        sb.synchronize()
        out["encode"] = (time.perf_counter() - t) / n


warm = {}
decode_loop(1, warm)
encode_loop(1, warm)
alone = {}
decode_loop(ITERS, alone)
encode_loop(ITERS, alone)
both = {}
t0 = time.perf_counter()
th = [threading.Thread(target=decode_loop, args=(ITERS, both)), threading.Thread(target=encode_loop, args=(ITERS, both))]
for t in th:
    t.start()
for t in th:
    t.join()
wall = (time.perf_counter() - t0) / ITERS
serial = alone["decode"] + alone["encode"]
print({"decode_alone_s": round(alone["decode"], 4), "encode_alone_s": round(alone["encode"], 4),
       "both_wall_s": round(wall, 4), "both_decode_s": round(both["decode"], 4), "both_encode_s": round(both["encode"], 4),
       "saved_frac_of_serial": round(1 - wall / serial, 4)}, flush=True)
