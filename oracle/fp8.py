"""OCP e4m3 ("e4m3fn") rounding and the per-position quantisation of the fp8 cross memory (TEST
INFRASTRUCTURE ONLY — see oracle/__init__.py).

The engine's opt-in fp8 cross memory (`wm_set_option("cross_fp8", 1)`, attn_xenc.hip `xquant8_kernel`) stores a
window's encoder output E as e4m3 codes of E[t] * (448 / amax_t) with one f32 scale amax_t / 448 per position
(amax_t = max_c |E[t][c]|; an all-zero row stores zeros with scale 0).  This restates it in numpy: products in
float32, round to nearest even onto the e4m3 grid (bias 7, 3 mantissa bits, subnormals below 2^-6, largest
finite 448), pinned against torch's float8_e4m3fn cast in tests/test_fp8_oracle.py.  The attention then sees
E_deq[t] = e4m3 value * scale_t; the tests decode the oracle on E_deq.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

E4M3_MAX = 448.0


def e4m3_round(x: np.ndarray) -> np.ndarray:
    """Round float32 values to the nearest e4m3 value (ties to even); |x| > 448 saturates (the engine never
    produces such inputs: its scaled rows have |x| <= 448 up to one float32 ulp)."""
    x = np.asarray(x, dtype=np.float32)
    a = np.abs(x).astype(np.float64)
    _, ex = np.frexp(np.where(a > 0, a, 1.0))
    e = np.maximum(ex - 1, -6)                           # exponent of the binade; subnormals share 2^-6's step
    step = np.ldexp(1.0, e - 3)
    q = np.round(a / step) * step                        # numpy rounds half to even
    q = np.minimum(q, E4M3_MAX)
    return np.copysign(q, x).astype(np.float32)


def e4m3_bits(v: np.ndarray) -> np.ndarray:
    """uint8 codes of values already on the e4m3 grid."""
    v = np.asarray(v, dtype=np.float64)
    s = (v < 0) | ((v == 0) & np.signbit(v))
    a = np.abs(v)
    _, ex = np.frexp(np.where(a > 0, a, 1.0))
    e = ex - 1
    normal = a >= 2.0 ** -6
    expf = np.where(normal, e + 7, 0)
    mant = np.where(normal, a / np.ldexp(1.0, e) * 8 - 8, a / 2.0 ** -9)
    mant = np.where(a > 0, mant, 0)
    return ((s.astype(np.uint8) << 7) | (expf.astype(np.uint8) << 3) | np.rint(mant).astype(np.uint8)).astype(np.uint8)


def quantize_rows(E: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """E [N][d] (bf16-valued float32) -> (codes uint8 [N][d], scale float32 [N], E_deq float32 [N][d])."""
    E = np.asarray(E, dtype=np.float32)
    amax = np.abs(E).max(axis=1).astype(np.float32)
    inv = np.where(amax > 0, np.float32(E4M3_MAX) / np.where(amax > 0, amax, np.float32(1)), np.float32(0))
    inv = inv.astype(np.float32)
    vals = e4m3_round((E * inv[:, None]).astype(np.float32))
    scale = (amax / np.float32(E4M3_MAX)).astype(np.float32)
    return e4m3_bits(vals), scale, (vals * scale[:, None]).astype(np.float32)
