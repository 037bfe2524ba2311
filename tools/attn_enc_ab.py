"""A/B of the encoder self-attention kernel forms (VLOG_AMD_ATTN_V = 2 | 3) at the bench's shape.

150 large-v3 windows are 3000 (window, head) pairs of T = 1500, head_dim 64; the tiny engine at B = 500 windows
(6 heads) launches the same 36,000 workgroups with the same per-workgroup work (only the qkv row stride differs).
Each form runs in its own child process (the form is read once per process); arms alternate on one box.  Prints
one JSON line per arm: ms per launch, TF/s (4 T^2 hd per pair), and a CRC of the output bytes (equal CRCs = the
forms agree bit for bit).

  python tools/attn_enc_ab.py [--forms 2,3,2,3] [--iters 30]
"""
import argparse
import json
import os
import subprocess
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(iters: int, B: int):
    sys.path.insert(0, ROOT)
    import torch
    from vlog_amd.dims import model_dims
    from vlog_amd.engine import GpuEngine
    from vlog_amd.weights import synthetic_state_dict
    dims = model_dims("tiny")
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=1, eot_after=40), 0)
    g = torch.Generator().manual_seed(0)
    qkv = (torch.randn(B, 1500, 3 * dims.n_state, generator=g)).to(torch.bfloat16).cuda()
    out = None
    for _ in range(3):
        out = eng.encoder_attention(qkv)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        out = eng.encoder_attention(qkv)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / iters
    flops = 4.0 * 1500 * 1500 * 64 * dims.n_head * B
    crc = zlib.crc32(out.view(torch.int16).cpu().numpy().tobytes())
    print(json.dumps(dict(form=os.environ.get("VLOG_AMD_ATTN_V"), B=B, ms=round(ms, 4),
                          tflops=round(flops / ms / 1e9, 1), crc=crc)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forms", default="2,3,2,3")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--B", type=int, default=500)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.iters, a.B)
        return
    for f in a.forms.split(","):
        env = dict(os.environ, VLOG_AMD_ATTN_V=f)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--iters", str(a.iters),
                            "--B", str(a.B)], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
