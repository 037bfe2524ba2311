"""Localise encoder-attention kernel errors with structured inputs (tools only)."""
import sys

import torch

sys.path.insert(0, ".")
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.weights import synthetic_state_dict  # noqa: E402

dims = model_dims("tiny")
eng = GpuEngine(dims, synthetic_state_dict(dims, seed=1, eot_after=40), 0)
H, d, T = dims.n_head, dims.n_state, 1500


def ref(x):
    q, k, v = x[0, :, 0].permute(1, 0, 2), x[0, :, 1].permute(1, 0, 2), x[0, :, 2].permute(1, 0, 2)
    o = torch.softmax((q @ k.transpose(-1, -2)) * 0.125, -1) @ v
    return o.permute(1, 0, 2).reshape(T, d)


def run(name, x):
    qkv = x.reshape(1, T, 3 * d).to(torch.bfloat16).cuda()
    xb = qkv.float().cpu().view(1, T, 3, H, 64)
    got = eng.encoder_attention(qkv).float().cpu()[0]
    r = ref(xb)
    e = (got - r).abs()
    print(f"{name:28s} max err {e.max():.4f} mean {e.mean():.5f} scale {r.abs().max():.4f}")
    return got, r


g = torch.Generator().manual_seed(0)
# 1. uniform attention (Q = 0): O = column means of V -> tests the P.V path alone
x = torch.zeros(1, T, 3, H, 64)
x[0, :, 2] = torch.randn(T, H, 64, generator=g)
got, r = run("Q=0, V random", x)
print(" got[0,:8]", got[0, :8].tolist())
print(" ref[0,:8]", r[0, :8].tolist())
# 2. V = key index (same for every hd): O = expected key index -> tests S/softmax
x = torch.randn(1, T, 3, H, 64, generator=g) * 0.5
x[0, :, 2] = (torch.arange(T).float() / T)[:, None, None].expand(T, H, 64)
got, r = run("V = key/T", x)
print(" got[0:4,0]", got[0:4, 0].tolist(), " ref", r[0:4, 0].tolist())
# 3. V one-hot on hd = key % 64, Q = 0
x = torch.zeros(1, T, 3, H, 64)
for k in range(T):
    x[0, k, 2, :, k % 64] = 1.0
got, r = run("Q=0, V onehot(key%64)", x)
print(" got[0,:16]", [round(v, 4) for v in got[0, :16].tolist()])
print(" ref[0,:16]", [round(v, 4) for v in r[0, :16].tolist()])
# 4. only the first 64 keys nonzero V, Q = 0
x = torch.zeros(1, T, 3, H, 64)
x[0, :64, 2] = torch.randn(64, H, 64, generator=g)
run("Q=0, V tile0 only", x)
x = torch.zeros(1, T, 3, H, 64)
x[0, 64:128, 2] = torch.randn(64, H, 64, generator=g)
run("Q=0, V tile1 only", x)
# 5. random
x = torch.randn(1, T, 3, H, 64, generator=g)
run("random", x)
