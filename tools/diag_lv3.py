"""Diagnostic (tools only): large-v3 greedy decode of 150 bench windows under engine knob variants; teacher-forced
oracle margins for a few windows per variant, and token agreement between variants.  Prints one JSON line per
variant.   usage: python tools/diag_lv3.py [windows...]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.decode import GenerateOptions  # noqa: E402
from oracle.model import OracleWhisper  # noqa: E402
from tests.parity_util import window_parity  # noqa: E402
from vlog_amd.audio import speech_like  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.tokenizer import Tokenizer  # noqa: E402
from vlog_amd.weights import round_bf16, synthetic_state_dict  # noqa: E402

W = 150
check = [int(a) for a in sys.argv[1:]] or [0, 85, 106, 128, 149]
dims = model_dims("large-v3")
sd = synthetic_state_dict(dims, seed=0, eot_after=110)
eng = GpuEngine(dims, sd, 0)
orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
del sd
x = np.concatenate([speech_like(30.0, i) for i in range(W)])
mel = eng.features(torch.from_numpy(x))
enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W)
tok = Tokenizer(dims, language="en")
prompt = list(tok.sot_sequence)
sup = list(tok.suppressed_tokens([-1]))
opt = GenerateOptions(suppress_tokens=sup, max_length=448)
encw = {w: enc[w].float().cpu().numpy() for w in check}
variants = [
    ("default", {}),
    ("ring_off", {"decode_ring_gemm": 0}),
    ("fuse_off", {"cross_attn_fuse": 0}),
    ("projected", {"cross_mode": 0}),
    ("plan0", {"decode_gemm_plan": 0}),
]
base = {"decode_ring_gemm": 1, "cross_attn_fuse": 1, "cross_mode": 1, "decode_gemm_plan": 1}
toks = {}
for name, kv in variants:
    for k, v in base.items():
        eng.set_option(k, v)
    for k, v in kv.items():
        eng.set_option(k, v)
    eng.reserve(W, W)
    eng.cross_kv(enc, 0)
    torch.cuda.synchronize()
    t = time.time()
    res, steps = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=448, check_every=8)
    dt = time.time() - t
    toks[name] = [r.tokens for r in res]
    rows = [window_parity(orc, encw[w], prompt, res[w], dims.specials, opt, w) for w in check]
    same = {v: sum(a == b for a, b in zip(toks[name], toks[v])) for v in toks}
    print(json.dumps({"variant": name, "s": round(dt, 3), "margins": {r.window: round(r.min_margin, 4) for r in rows},
                      "tie_margins": {r.window: [round(r.min_margin_rule_tie, 4), r.worst_step, round(r.worst_gap, 4)] for r in rows},
                      "identical": {r.window: r.identical for r in rows}, "same_tokens_as": same}), flush=True)
