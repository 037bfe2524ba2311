"""Diagnostic (round 5): determinism and split-schedule identity of the folded-LayerNorm decode (decode_ln_fold)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import mel as omel
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.engine import GpuEngine
from vlog_amd.weights import synthetic_state_dict

W = 40
dims = model_dims("tiny")
eng = GpuEngine(dims, synthetic_state_dict(dims, seed=11, eot_after=40), 0)
x = np.concatenate([speech_like(30.0, 500 + i) for i in range(W)])
enc = eng.encode(torch.from_numpy(omel.log_mel(x, dims.n_mels)).cuda(), [3000 * i for i in range(W)], [3000] * W)
eng.reserve(W, 5 * W)
eng.cross_kv(enc, 0)
st = dims.specials
prompt = [st.sot, st.lang_token("en"), st.transcribe]
sup = [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]


def run(fold, split, graph=1):
    eng.set_option("decode_ln_fold", fold)
    eng.set_option("decode_split", split)
    eng.set_option("decode_graph", graph)
    res, steps = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=120)
    eng.set_option("decode_split", 0)
    eng.set_option("decode_graph", 1)
    return [tuple(r.tokens) for r in res], [r.cum_logprob for r in res]


base = {}
for name, args in [("fold", (1, 0)), ("fold_again", (1, 0)), ("fold_split", (1, 1)), ("fold_eager", (1, 0, 0)),
                   ("fold_split_eager", (1, 1, 0)), ("nofold", (0, 0)), ("nofold_split", (0, 1))]:
    t, c = run(*args)
    base[name] = (t, c)
    ref = base["fold"] if name.startswith("fold") else base.get("nofold", (t, c))
    same = sum(a == b for a, b in zip(t, ref[0]))
    dc = max(abs(a - b) for a, b in zip(c, ref[1]))
    print(name, "windows identical to", "fold" if name.startswith("fold") else "nofold", same, "/", W, "max dcum", dc, flush=True)
t0, c0 = base["nofold"]
t1, c1 = base["fold"]
print("fold vs nofold identical windows", sum(a == b for a, b in zip(t0, t1)), "max dcum", max(abs(a - b) for a, b in zip(c0, c1)))
