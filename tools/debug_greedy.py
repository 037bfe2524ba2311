import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from oracle import mel as omel
from oracle.decode import GenerateOptions, generate_one, apply_rules, log_softmax
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.engine import GpuEngine
from vlog_amd.weights import round_bf16, synthetic_state_dict
dims = model_dims("tiny"); st = dims.specials
sd = synthetic_state_dict(dims, seed=3, eot_after=60)
eng = GpuEngine(dims, sd, 0)
o32 = OracleWhisper(round_bf16(sd), dims, np.float32)
obf = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
W = 6
x = np.concatenate([speech_like(30.0, 100 + i) for i in range(W)])
feats = omel.log_mel(x, dims.n_mels)
enc = eng.encode(torch.from_numpy(feats).cuda(), [3000 * i for i in range(W)], [3000] * W)
eng.reserve(W, W); eng.cross_kv(enc, 0)
prompt = [st.sot, st.lang_token("en"), st.transcribe]
sup = [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]
res, _ = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=120)
encf = enc.float().cpu().numpy()
for w in range(W):
    r = generate_one(obf, obf.cross_kv(encf[w:w+1]), prompt, st, GenerateOptions(suppress_tokens=sup, max_length=120))
    g = res[w].tokens
    if r.tokens == g:
        print(w, "identical", len(g)); continue
    k = next(i for i in range(min(len(g), len(r.tokens))) if g[i] != r.tokens[i]) if any(a != b for a, b in zip(g, r.tokens)) else min(len(g), len(r.tokens))
    print(w, "diverge at", k, "gpu", g[k:k+3], "orc", r.tokens[k:k+3], "lens", len(g), len(r.tokens))
    seq = np.array([prompt + g[:k]])
    lg_gpu, _ = eng.forward([w], seq)
    lg_bf, _ = obf.decode(seq, obf.cross_kv(encf[w:w+1]))
    lg_32, _ = o32.decode(seq, o32.cross_kv(encf[w:w+1]))
    a, b, c = lg_gpu[0, -1].cpu().numpy(), lg_bf[0, -1], lg_32[0, -1]
    print("  |gpu-bf| max", np.abs(a - b).max(), " |gpu-f32| max", np.abs(a - c).max(), " |bf-f32|", np.abs(b - c).max())
    for name, v in (("gpu", a), ("bf", b), ("f32", c)):
        m = apply_rules(v, g[:k], st, sup, True, 50)
        lp = log_softmax(m); top = np.argsort(-lp)[:3]
        print("  ", name, top, lp[top])
