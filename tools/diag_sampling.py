"""Diagnostic (tools only): a sampled GPU hypothesis vs the oracle, step by step — teacher-forced logits on the GPU
(wm_forward) and in the oracle, and the Gumbel keys of the engine's noise, around the worst step."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import mel as omel  # noqa: E402
from oracle.decode import apply_rules, gumbel_noise, log_softmax  # noqa: E402
from oracle.model import OracleWhisper  # noqa: E402
from vlog_amd.audio import speech_like  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.weights import round_bf16, synthetic_state_dict  # noqa: E402

dims = model_dims("tiny")
sd = synthetic_state_dict(dims, seed=3, eot_after=60)
eng = GpuEngine(dims, sd, 0)
orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
W = 4
x = np.concatenate([speech_like(30.0, 800 + i) for i in range(W)])
feats = omel.log_mel(x, dims.n_mels)
enc = eng.encode(torch.from_numpy(feats).cuda(), [3000 * i for i in range(W)], [3000] * W)
eng.reserve(W, 16)
eng.cross_kv(enc, 0)
st = dims.specials
prompt = [st.sot, st.lang_token("en"), st.transcribe]
sup = [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]
T, nh, seed = 1.0, 3, 11
res, _ = eng.generate(list(range(W)), [prompt] * W, temperature=T, num_hypotheses=nh, seed=seed, suppress_tokens=sup,
                      max_length=120)
w = 2
toks = res[w].tokens
print("window", w, "len", len(toks), "score", res[w].score)
seqt = np.array([prompt + toks])
gl, _ = eng.forward([w], seqt)
gl = gl[0].cpu().numpy()
encf = enc.float().cpu().numpy()
cross = orc.cross_kv(encf[w: w + 1])
ol, _ = orc.decode(seqt, cross)
ol = ol[0]
P = len(prompt)
for j in range(nh):
    worst = []
    for i, t in enumerate(toks):
        xo = apply_rules(ol[P - 1 + i], toks[:i], st, sup, True, 50, True)
        xg = apply_rules(gl[P - 1 + i], toks[:i], st, sup, True, 50, True)
        g = gumbel_noise(seed, w * nh + j, i, xo.shape[0])
        ko, kg = xo / T + g, xg / T + g
        worst.append((float(ko[t] - ko.max()), float(kg[t] - kg.max()), i, int(np.argmax(ko)), int(np.argmax(kg)), t,
                      float(np.abs(gl[P - 1 + i] - ol[P - 1 + i]).max())))
    worst.sort()
    print("hyp", j, "worst (oracle-key margin, gpu-forward-key margin, step, oracle argmax, gpu-forward argmax, token, max|dlogit|):")
    for r in worst[:4]:
        print("   ", r)
