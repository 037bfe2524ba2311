"""The small-M decoder GEMM (gemm_dec.hip gemv_dec_kernel: passes of <= 32 rows — one window's beam, a handful
of windows) against the CPU oracle and against the general decoder GEMM routes, on the margin-planted models
(decisive logits, so the token comparisons are exact gates): greedy over 8 windows (8 rows) and beam 5 over
4 windows (20 rows) and over 1 window (5 rows: the worker's sequential call)."""
import numpy as np
import pytest
import torch

from oracle.decode import GenerateOptions, beam_many
from oracle.model import OracleWhisper
from tests.parity_util import assert_gates, gate_windows
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["tiny", "small"])
def setup(request):
    from vlog_amd.engine import GpuEngine
    dims = model_dims(request.param)
    sd = synthetic_state_dict(dims, seed=0, plant="margin")
    eng = GpuEngine(dims, sd, 0)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
    W = 8
    x = np.concatenate([speech_like(30.0, 40 + i) for i in range(W)])
    mel = eng.features(torch.from_numpy(x))
    enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W)
    tok = Tokenizer(dims, language="en")
    return dims, eng, orc, enc, tok


def _gen(eng, enc, tok, ws, beam, gemv, gemv_ln=1, ln_fc2=0):
    eng.set_option("decode_gemv", gemv)
    eng.set_option("decode_gemv_ln", gemv_ln)
    eng.set_option("decode_gemv_ln_fc2", ln_fc2)
    eng.set_option("cross_mode", 0 if beam > 1 else 1)
    try:
        eng.reserve(enc.shape[0], enc.shape[0] * beam)
        eng.cross_kv(enc, 0)
        res, _ = eng.generate(ws, [list(tok.sot_sequence)] * len(ws), beam_size=beam,
                              suppress_tokens=list(tok.suppressed_tokens([-1])), max_length=448)
    finally:
        eng.set_option("decode_gemv", 1)
        eng.set_option("decode_gemv_ln", 1)
        eng.set_option("decode_gemv_ln_fc2", 0)
        eng.set_option("cross_mode", 1)
    return res


@pytest.mark.parametrize("ws,beam", [(list(range(8)), 1), ([0, 3, 5, 7], 5), ([6], 5)], ids=["greedy8", "beam5x4", "beam5x1"])
def test_gemv_route_vs_oracle_and_general_route(setup, ws, beam):
    dims, eng, orc, enc, tok = setup
    a = _gen(eng, enc, tok, ws, beam, 1)
    b = _gen(eng, enc, tok, ws, beam, 0)
    c = _gen(eng, enc, tok, ws, beam, 1, gemv_ln=0)        # LayerNorm combine launches instead of the fused form
    d = _gen(eng, enc, tok, ws, beam, 1, ln_fc2=1)         # opt-in: fc2 -> next layer's ln1 fused as well
    assert [r.tokens for r in a] == [r.tokens for r in b] == [r.tokens for r in c] == [r.tokens for r in d]
    # the fused LayerNorm merges per-tile statistics (another summation order): f32-rounding agreement
    assert max(abs(x.score - y.score) for x, y in zip(a, c)) < 2e-3
    assert max(abs(x.score - y.score) for x, y in zip(a, d)) < 2e-3
    encf = enc.float().cpu().numpy()
    opt = GenerateOptions(beam_size=beam, suppress_tokens=list(tok.suppressed_tokens([-1])), max_length=448)
    res = {w: r for w, r in zip(ws, a)}
    g = gate_windows(orc, lambda w: encf[list(w)], list(tok.sot_sequence), res, dims.specials, opt, tok, windows=ws)
    assert_gates(g)
    if beam > 1:
        refs = beam_many(orc, orc.cross_kv(encf[ws]), list(tok.sot_sequence), dims.specials, opt)
        assert [r.tokens for r in refs] == [r.tokens for r in a]


def test_gemv_check_fused_layernorm_statistics():
    """tools/gemv_check (built in-tree by the library's Makefile): the small-M residual producer's per-tile row
    statistics (sum, and sum of squares about the tile mean) and the LayerNorm-consuming operand, in isolation
    against a CPU reference, with canary guards around every buffer — including a residual with a common offset of
    1000 (|mean| / std ~ 580), where a one-pass E[x^2] - mean^2 variance would lose its digits in f32."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "gemv_check")
    if not os.path.exists(exe):
        pytest.skip("tools/gemv_check not built (make -C vlog_amd/csrc ../../tools/gemv_check)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0 and "all ok" in r.stdout, r.stdout + r.stderr
