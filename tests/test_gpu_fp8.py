"""Opt-in fp8 cross memory (wm_set_option "cross_fp8"): the window slots hold the encoder output
as OCP e4m3 codes with one scale per position, and the factored cross-attention streams half the bytes.

  * the quantisation kernel is bit-exact with oracle/fp8.py (itself pinned to torch's float8_e4m3fn cast);
  * decoding in fp8 mode is compared with the oracle run on the DEQUANTISED encoder output (the values the
    kernel actually attends over), with the same generate-boundary checks as the bf16 configs
    (tests/parity_util.py) — tiny (8 windows) here, large-v3 at the bench size in tests/test_gpu_configs.py.
"""
import numpy as np
import pytest
import torch

from oracle import fp8
from oracle.decode import GenerateOptions
from oracle.model import OracleWhisper
from tests.parity_util import record, window_parity
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu


def test_quantize_kernel_bitexact():
    """tiny (n_state 384); the large-v3 instantiation (1280) is checked in tests/test_gpu_configs.py."""
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=0), 0)
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(300, dims.n_state, generator=g) * torch.rand(300, 1, generator=g) * 30).bfloat16()
    x[5] = 0
    x[6, :7] = -0.0
    codes, scale = eng.cross_fp8_quantize(x.cuda())
    rc, rs, _ = fp8.quantize_rows(x.float().numpy())
    assert np.array_equal(scale.cpu().numpy(), rs)
    assert np.array_equal(codes.cpu().numpy(), rc)


def test_fp8_decode_tiny_vs_oracle():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=3, eot_after=60)
    eng = GpuEngine(dims, sd, 0)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
    W = 8
    x = np.concatenate([speech_like(30.0, 900 + i) for i in range(W)])
    mel = eng.features(torch.from_numpy(x))
    enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W)
    tok = Tokenizer(dims, language="en")
    prompt, sup = list(tok.sot_sequence), list(tok.suppressed_tokens([-1]))
    eng.set_option("cross_fp8", 1)
    try:
        eng.reserve(W, W)
        eng.cross_kv(enc, 0)
        res, _ = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=448)
    finally:
        eng.set_option("cross_fp8", 0)
    opt = GenerateOptions(suppress_tokens=sup, max_length=448)
    rows = []
    for w in range(W):
        deq = fp8.quantize_rows(enc[w].float().cpu().numpy())[2]
        rows.append(window_parity(orc, deq, prompt, res[w], dims.specials, opt, w, eps=0.02))
    record("tiny fp8 cross memory 8 windows", rows)
    for r in rows:
        assert r.min_margin_rule_tie >= -0.02, (r.window, r.min_margin_rule_tie)
        assert abs(r.no_speech_gpu - r.no_speech_oracle) < 1e-3
