"""Scheduling knobs must not change results: the two-slice decode (decoder rows split over two streams), the
fused cross-attention (cq split-K combine + key-split combine folded into the attention kernel) and its
persistent grid form give bit-identical tokens, scores and no-speech probabilities to the plain schedule,
for greedy and beam search.  Runs through the C-ABI on the MI355X."""
import numpy as np
import pytest
import torch

from oracle import mel as omel
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

W = 40
_ENC = []      # the fixture's encoder output (tests that switch the cross form re-fill the slots from it)


@pytest.fixture(scope="module")
def batch():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=11, eot_after=40)
    eng = GpuEngine(dims, sd, 0)
    x = np.concatenate([speech_like(30.0, 500 + i) for i in range(W)])
    feats = omel.log_mel(x, dims.n_mels)
    enc = eng.encode(torch.from_numpy(feats).cuda(), [3000 * i for i in range(W)], [3000] * W)
    eng.reserve(W, 5 * W)
    eng.cross_kv(enc, 0)
    _ENC.append(enc)
    return dims, eng


def _run(eng, dims, split, opts=(), windows=W, **kw):
    st = dims.specials
    eng.set_option("decode_split", split)
    for k, v in opts:
        eng.set_option(k, v)
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    sup = [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]
    res, steps = eng.generate(list(range(windows)), [prompt] * windows, suppress_tokens=sup, max_length=120, **kw)
    eng.set_option("decode_split", 0)                 # back to the defaults
    eng.set_option("cross_attn_fuse", 1)
    eng.set_option("cross_attn_blocks", 0)
    eng.set_option("cross_attn_snake", 0)
    eng.set_option("cross_attn_keep", 0)
    eng.set_option("decode_gemm_plan", 1)          # also restores the preset's column widths
    eng.set_option("cross_mfma_fuse", 0)
    return res, steps


def _same(a, sa, b, sb):
    assert sa == sb
    for ra, rb in zip(a, b):
        assert ra.tokens == rb.tokens
        assert ra.score == rb.score and ra.cum_logprob == rb.cum_logprob
        assert ra.no_speech_prob == rb.no_speech_prob


@pytest.mark.parametrize("kw", [dict(), dict(beam_size=5, patience=1.0)], ids=["greedy", "beam5"])
@pytest.mark.parametrize("opts", [(("cross_attn_fuse", 0),), (("cross_attn_blocks", 512),),
                                  (("cross_attn_fuse", 3), ("cross_attn_blocks", 512))],
                         ids=["unfused", "persistent", "combine-fused-persistent"])
def test_cross_attention_forms_bit_identical(batch, kw, opts):
    dims, eng = batch
    a, sa = _run(eng, dims, 0, **kw)
    b, sb = _run(eng, dims, 0, opts=opts, **kw)
    _same(a, sa, b, sb)


@pytest.mark.parametrize("windows", [2, W])
def test_mfma_beam_combine_fused_bit_identical(batch, windows):
    """Projected form, beam groups on the matrix-core cross-attention: the key-split merge done by the last-arriving
    split inside the kernel (cross_mfma_fuse=1) vs the separate combine kernel: same arithmetic and order, so the
    same tokens, scores and no-speech probabilities (2 windows: 16 key splits; 40 windows: 3)."""
    dims, eng = batch
    kw = dict(beam_size=5, patience=1.0)
    eng.set_option("cross_mode", 0)             # the product's form for beam groups (transcribe.py)
    try:
        eng.cross_kv(_ENC[0], 0)
        a, sa = _run(eng, dims, 0, windows=windows, **kw)
        b, sb = _run(eng, dims, 0, opts=(("cross_mfma_fuse", 1),), windows=windows, **kw)
    finally:
        eng.set_option("cross_mode", 1)
        eng.cross_kv(_ENC[0], 0)
    _same(a, sa, b, sb)
    assert sum(len(r.tokens) for r in a) > windows * 5


@pytest.mark.parametrize("kw", [dict(), dict(beam_size=5, patience=1.0)], ids=["greedy", "beam5"])
def test_ring_columns_and_snake_order_bit_identical(batch, kw):
    """64-column ring-GEMM tiles and the layer-alternating cross-attention item order change only the schedule:
    each output keeps its K summation order and each attention item its arithmetic."""
    dims, eng = batch
    rows64 = (("decode_gemm.qkv", 64), ("decode_gemm.fc1", 64), ("decode_gemm.out", 32))
    cols32 = tuple(("decode_gemm_cols." + pj, 32) for pj in ("qkv", "fc1", "out"))
    a, sa = _run(eng, dims, 0, opts=rows64 + cols32, **kw)
    b, sb = _run(eng, dims, 0, opts=rows64 + (("decode_gemm_cols.qkv", 64), ("decode_gemm_cols.fc1", 64),
                                              ("decode_gemm_cols.out", 64), ("cross_attn_snake", 1),
                                              ("cross_attn_keep", W // 2)), **kw)
    _same(a, sa, b, sb)
    assert sum(len(r.tokens) for r in a) > W * 5


@pytest.mark.parametrize("kw", [dict(), dict(beam_size=5, patience=1.0)], ids=["greedy", "beam5"])
def test_split_decode_bit_identical(batch, kw):
    dims, eng = batch
    a, sa = _run(eng, dims, 1, **kw)
    b, sb = _run(eng, dims, 0, **kw)
    assert sa == sb
    for ra, rb in zip(a, b):
        assert ra.tokens == rb.tokens
        assert ra.score == rb.score and ra.cum_logprob == rb.cum_logprob
        assert ra.no_speech_prob == rb.no_speech_prob
    assert sum(len(r.tokens) for r in a) > W * 5


@pytest.mark.parametrize("kw", [dict(), dict(beam_size=5, patience=1.0),
                                dict(temperature=0.6, num_hypotheses=5, seed=7)], ids=["greedy", "beam5", "sampling"])
def test_step_graph_replay_bit_identical(batch, kw):
    """Decode steps replayed from one captured HIP graph (decode_graph=1, the default) vs launched eagerly: the
    same tokens, scores and no-speech probabilities (sampling keys its Gumbel noise on the device-side step)."""
    dims, eng = batch
    a, sa = _run(eng, dims, 0, opts=(("decode_graph", 0),), **kw)
    eng.set_option("decode_graph", 1)
    b, sb = _run(eng, dims, 0, **kw)
    _same(a, sa, b, sb)
    assert sum(len(r.tokens) for r in a) > W * 5


def test_unknown_option_raises(batch):
    _, eng = batch
    with pytest.raises(RuntimeError, match="unknown option"):
        eng.set_option("no_such_knob", 1)
    with pytest.raises(RuntimeError, match="32 or 64"):
        eng.set_option("decode_gemm_cols.fc1", 48)
    with pytest.raises(RuntimeError, match="unknown projection"):
        eng.set_option("decode_gemm_cols.nope", 64)
