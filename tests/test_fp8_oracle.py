"""CPU: the e4m3 restatement (oracle/fp8.py) pinned against torch's float8_e4m3fn cast (round to nearest even),
and the per-position quantisation of the fp8 cross memory."""
import numpy as np
import torch

from oracle import fp8


def test_e4m3_round_and_bits_match_torch():
    rng = np.random.default_rng(0)
    x = np.concatenate([
        rng.standard_normal(20000).astype(np.float32) * 50,
        rng.standard_normal(5000).astype(np.float32) * 0.01,             # subnormal range
        np.array([0.0, -0.0, 448.0, -448.0, 2.0 ** -9, 2.0 ** -10, 3 * 2.0 ** -10, 1.0625, 1.1875, 240.0, 232.0],
                 np.float32),
    ])
    x = np.clip(x, -448, 448)
    ours = fp8.e4m3_round(x)
    t = torch.from_numpy(x).to(torch.float8_e4m3fn)
    assert np.array_equal(ours, t.float().numpy())
    assert np.array_equal(fp8.e4m3_bits(ours), t.view(torch.uint8).numpy())


def test_quantize_rows():
    rng = np.random.default_rng(1)
    E = (rng.standard_normal((64, 1280)) * rng.uniform(0.1, 20, (64, 1))).astype(np.float32)
    E[3] = 0.0
    E = torch.from_numpy(E).bfloat16().float().numpy()
    codes, scale, deq = fp8.quantize_rows(E)
    assert codes.dtype == np.uint8 and codes.shape == E.shape and scale.shape == (64,)
    assert scale[3] == 0 and np.all(deq[3] == 0) and np.all(codes[3] == 0)
    # every row's largest magnitude maps to 448 (code 0x7E / 0xFE)
    nz = np.arange(64) != 3
    assert np.all((codes[nz] & 0x7F).max(axis=1) == 0x7E)
    rel = np.abs(deq - E) / np.maximum(np.abs(E).max(axis=1, keepdims=True), 1e-30)
    assert rel.max() <= 2.0 ** -4 + 1e-6          # half a step of the top binade, relative to the row max
