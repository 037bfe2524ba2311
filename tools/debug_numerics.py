import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from oracle import mel as omel
import oracle.model as om
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.engine import GpuEngine
from vlog_amd.weights import round_bf16, synthetic_state_dict
dims = model_dims("tiny"); st = dims.specials
sd = synthetic_state_dict(dims, seed=3, eot_after=60)
eng = GpuEngine(dims, sd, 0)
w = round_bf16(sd)
feats = omel.log_mel(speech_like(30.0, 102), dims.n_mels)
enc = eng.encode(torch.from_numpy(feats).cuda(), [0], [3000])
eng.reserve(2, 2); eng.cross_kv(enc, 0)
encf = enc.float().cpu().numpy()
seq = np.array([[st.sot, st.lang_token("en"), st.transcribe] + list(range(700, 720))])
g = eng.forward([0], seq)[0][0].cpu().numpy()
variants = {"f32": dict(bf16_acts=False), "bf16": dict(bf16_acts=True)}
for name, kw in variants.items():
    o = OracleWhisper(w, dims, np.float32, **kw)
    r = o.decode(seq, o.cross_kv(encf))[0][0]
    d = np.abs(g - r).max(-1)
    print(name, "max|gpu-oracle| per position", np.round(d, 4))
# oracle with f64 accumulation but bf16 rounding points
o = OracleWhisper(w, dims, np.float64, bf16_acts=True)
r = o.decode(seq, o.cross_kv(encf))[0][0]
print("bf16/f64acc", np.round(np.abs(g - r).max(-1), 4))
print("logit scale", np.abs(g).max())
