"""Decoder passes of >= decode_gemm_big_rows rows (beam groups of many windows; engine.cpp decoder_layer): the
64-row ring-GEMM route at its two LDS budgets ("decode_gemm_big_lds" 72 = two resident blocks per CU, the default,
and 144 = one) must give the same bits — the ring depth never changes a row's K summation order — and the same
tokens as the route below the threshold.  Beam 5 over 110 windows of the margin-planted tiny model (550 rows), over
64 (320 rows) and over 40 (200 rows, above the default threshold of 161).  The 8-wave plan ("decode_gemm_big128":
128 x 64 / 128 x 128 / 64 x 64 tiles of 8 waves) walks every row's K in the same order, so it must give the same
bits too."""
import numpy as np
import pytest
import torch

from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

W = 110


@pytest.fixture(scope="module")
def setup():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=0, plant="margin"), 0)
    x = np.concatenate([speech_like(30.0, 70 + i) for i in range(W)])
    mel = eng.features(torch.from_numpy(x))
    enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W)
    return dims, eng, enc, Tokenizer(dims, language="en")


def _beam(eng, enc, tok, n=W, **opts):
    old = {k: eng.option(k) for k in opts}
    for k, v in opts.items():
        eng.set_option(k, v)
    eng.set_option("cross_mode", 0)
    try:
        eng.reserve(W, W * 5)
        eng.cross_kv(enc, 0)
        res, _ = eng.generate(list(range(n)), [list(tok.sot_sequence)] * n, beam_size=5,
                              suppress_tokens=list(tok.suppressed_tokens([-1])), max_length=448)
    finally:
        for k, v in old.items():
            eng.set_option(k, v)
        eng.set_option("cross_mode", 1)
    return res


def test_big_rows_lds_budgets_bit_identical(setup):
    dims, eng, enc, tok = setup
    assert eng.option("decode_gemm_big_lds") == 72 and eng.option("decode_gemm_big_rows") == 161
    for n in (W, 64, 40):
        a = _beam(eng, enc, tok, n=n, decode_gemm_big_lds=72, decode_gemm_big128=0)     # the 4-wave route
        b = _beam(eng, enc, tok, n=n, decode_gemm_big_lds=144, decode_gemm_big128=0)
        c = _beam(eng, enc, tok, n=n, decode_gemm_big_rows=0)    # the route below the threshold (150-row plan)
        # the 8-wave plan on every big pass: with fc2 over its whole K the same bits; with fc2's K in ranges (its default)
        # the slabs are summed by the combine, so the same tokens and scores to f32 rounding
        d = _beam(eng, enc, tok, n=n, decode_gemm_big128=161, decode_gemm_big_fc2_kr=0)
        e = _beam(eng, enc, tok, n=n, decode_gemm_big128=161)
        assert [r.tokens for r in a] == [r.tokens for r in b], n
        assert [r.score for r in a] == [r.score for r in b], n  # bit for bit
        assert [r.tokens for r in a] == [r.tokens for r in d], n
        assert [r.score for r in a] == [r.score for r in d], n  # bit for bit
        assert [r.tokens for r in a] == [r.tokens for r in e], n
        assert max(abs(x.score - y.score) for x, y in zip(a, e)) < 2e-3, n
        assert [r.tokens for r in a] == [r.tokens for r in c], n
        assert max(abs(x.score - y.score) for x, y in zip(a, c)) < 2e-3, n
        if n == W:
            full = a
        else:
            assert [r.tokens for r in a] == [r.tokens for r in full[:n]], n


def test_big_lds_option_validation(setup):
    _, eng, _, _ = setup
    with pytest.raises(Exception):
        eng.set_option("decode_gemm_big_lds", 100)
    assert eng.option("decode_gemm_big_lds") == 72
