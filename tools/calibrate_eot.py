"""Sweep the synthetic-weights <|endoftext|> plant (vlog_amd/weights.py plant_eot) on the GPU and print the
mean greedy tokens per 30 s window, so bench.py's --eot-after gives a speech-like token count."""
import sys
import numpy as np
import torch
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.engine import GpuEngine
from vlog_amd.tokenizer import Tokenizer
import vlog_amd.weights as W

name = sys.argv[1]
kappa = float(sys.argv[2])
W.EOT_KAPPA = kappa
dims = model_dims(name)
st = dims.specials
tok = Tokenizer(dims, language="en")
Wn = 16
x = np.concatenate([speech_like(30.0, i) for i in range(Wn)])
for ea in [int(v) for v in sys.argv[3:]]:
    eng = GpuEngine(dims, W.synthetic_state_dict(dims, 0, eot_after=ea), 0)
    mel = eng.features(torch.from_numpy(x))
    enc = eng.encode(mel, [3000 * i for i in range(Wn)], [3000] * Wn)
    eng.reserve(Wn, Wn)
    eng.cross_kv(enc, 0)
    res, steps = eng.generate(list(range(Wn)), [[st.sot, st.lang_token("en"), st.transcribe]] * Wn,
                              suppress_tokens=tok.suppressed_tokens([-1]), max_length=448)
    lens = [len(r.tokens) for r in res]
    print(name, kappa, ea, "mean tokens", np.mean(lens), "min", min(lens), "max", max(lens), flush=True)
    del eng
    torch.cuda.empty_cache()
