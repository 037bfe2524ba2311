"""Factored cross-attention (attention over the encoder output, csrc/attn_xenc.hip; the engine default) against
the projected cross-KV path (csrc/attn_dec.hip, `cross_mode` 0) and the f32 oracle, through the C-ABI.

The two forms are the same arithmetic reassociated (q.(E Wk^T) = (Wk^T q).E, P (E Wv^T + bv) = (P E) Wv^T + bv),
so they agree to bf16 rounding noise: teacher-forced logits, alignment-head attention and no-speech
probabilities within the tolerances below, and the same greedy / beam tokens on (almost) every window.  The
model sizes cover every kernel instantiation: tiny (4 waves x 96 columns), base (8 x 64), small (8 x 96) and,
without the oracle, large-v3 (8 x 160, the bench configuration)."""
import numpy as np
import pytest
import torch

from oracle import mel as omel
from oracle.decode import GenerateOptions
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.weights import round_bf16, synthetic_state_dict
from tests.parity_util import window_parity

pytestmark = pytest.mark.gpu


def _sup(st):
    return [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]


def _engine(name, seed, W, eot_after=40):
    from vlog_amd.engine import GpuEngine
    dims = model_dims(name)
    sd = synthetic_state_dict(dims, seed=seed, eot_after=eot_after)
    eng = GpuEngine(dims, sd, 0)
    x = np.concatenate([speech_like(30.0, 900 + seed * 10 + i) for i in range(W)])
    feats = omel.log_mel(x, dims.n_mels)
    enc = eng.encode(torch.from_numpy(feats).cuda(), [3000 * i for i in range(W)], [3000] * W)
    return dims, sd, eng, enc


def _both(eng, enc, W, n_hyp, fn):
    """fn() under the projected (0) and factored (1) cross-attention; the engine is left in factored mode."""
    out = {}
    for mode in (0, 1):
        eng.set_option("cross_mode", mode)
        eng.reserve(W, n_hyp)
        eng.cross_kv(enc, 0)
        out[mode] = fn()
    return out[0], out[1]


@pytest.fixture(scope="module", params=["tiny", "base", "small"])
def small_models(request):
    W = 4
    dims, sd, eng, enc = _engine(request.param, 7, W)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32)
    return dims, eng, enc, orc, W


def test_factored_logits_match_projected_and_oracle(small_models):
    dims, eng, enc, orc, W = small_models
    st = dims.specials
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe] + list(range(700, 760))] * 2)
    a, b = _both(eng, enc, W, 8, lambda: eng.forward([1, 3], toks)[0].cpu().numpy())
    encf = enc.float().cpu().numpy()
    scale = max(np.abs(a).max(), 1.0)
    assert np.abs(a - b).max() < 0.02 * scale, np.abs(a - b).max()
    for i, w in enumerate((1, 3)):
        ref, _ = orc.decode(toks[i:i + 1], orc.cross_kv(encf[w:w + 1]))
        assert np.abs(b[i] - ref[0]).max() < 0.02 * np.abs(ref).max() + 1e-3


def test_factored_alignment_capture(small_models):
    """Alignment-head probabilities: raw scores from the attention kernel, normalised by the split merge."""
    dims, eng, enc, orc, W = small_models
    st = dims.specials
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe, st.no_timestamps] + list(range(1000, 1030)) + [st.eot]])
    heads = dims.default_alignment_heads()
    a, b = _both(eng, enc, W, 8, lambda: eng.forward([2], toks, align_heads=heads)[1][0].cpu().numpy())
    assert np.allclose(b.sum(-1), 1.0, atol=1e-4)
    assert np.abs(a - b).max() < 2e-3
    _, _, cw = orc.decode(toks, orc.cross_kv(enc.float().cpu().numpy()[2:3]), return_cross_attn=True)
    ref = np.stack([cw[l][0, h] for l, h in heads], 1)
    assert np.abs(b - ref).max() < 2e-3


@pytest.mark.parametrize("mode", [0, 1], ids=["projected", "factored"])
def test_teacher_forced_mfma_cross_attention(small_models, mode):
    """The alignment pass's matrix-core cross-attention (attn_dec.hip cross_tf_kernel, option cross_tf) against the
    decode path's kernels of the same form and the f32 oracle: three windows x 150 rows (two 128-row tiles per
    window, the second partial), every alignment head captured, every other head on the one-pass form.  In the
    factored form the pass first projects each layer's K/V panels of its windows (wm_cross_kv's GEMM, one layer).
    Probabilities (f32, exactly normalised by the kernel's first pass) within 2e-3 of the oracle, logits within
    2 % of the scale."""
    dims, eng, enc, orc, W = small_models
    st = dims.specials
    heads = dims.default_alignment_heads()
    S = 150
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe, st.no_timestamps] +
                     list(range(2000 + 37 * i, 2000 + 37 * i + S - 5)) + [st.eot] for i in range(3)])
    eng.set_option("cross_mode", mode)
    eng.reserve(W, 8)
    eng.cross_kv(enc, 0)
    out = {}
    try:
        for tf in (1, 0):
            eng.set_option("cross_tf", tf)
            lg, at = eng.forward([0, 3, 1], toks, align_heads=heads)
            out[tf] = (lg.cpu().numpy(), at.cpu().numpy())
    finally:
        eng.set_option("cross_tf", 1)
        eng.set_option("cross_mode", 1)
        eng.reserve(W, 8)
        eng.cross_kv(enc, 0)
    (la, aa), (lb, ab) = out[1], out[0]
    assert np.all(np.isfinite(aa)) and np.allclose(aa.sum(-1), 1.0, atol=1e-4)
    assert np.abs(aa - ab).max() < 2e-3, np.abs(aa - ab).max()
    assert np.abs(la - lb).max() < 0.02 * max(np.abs(lb).max(), 1.0)
    encf = enc.float().cpu().numpy()
    for i, w in enumerate((0, 3, 1)):
        ref, _, cw = orc.decode(toks[i:i + 1], orc.cross_kv(encf[w:w + 1]), return_cross_attn=True)
        r = np.stack([cw[l][0, h] for l, h in heads], 1)
        assert np.abs(aa[i] - r).max() < 2e-3
        assert np.abs(la[i] - ref[0]).max() < 0.02 * np.abs(ref).max() + 1e-3


@pytest.mark.parametrize("kw", [dict(), dict(beam_size=5, patience=1.0)], ids=["greedy", "beam5"])
def test_factored_generate_matches_projected(small_models, kw):
    dims, eng, enc, orc, W = small_models
    st = dims.specials
    prompt = [st.sot, st.lang_token("en"), st.transcribe]

    def run():
        return eng.generate(list(range(W)), [prompt] * W, suppress_tokens=_sup(st), max_length=100, **kw)

    (ra, sa), (rb, sb) = _both(eng, enc, W, 5 * W, run)
    same = sum(x.tokens == y.tokens for x, y in zip(ra, rb))
    encf = enc.float().cpu().numpy()
    if kw:
        # beam search on random weights: the beams of near-tied hypotheses can part on bf16 noise between the two
        # forms (tools/diag_xattn_beam.py: tiny, 2 of 4 windows parted, one of them onto a sequence the oracle scores
        # HIGHER than its own beam result; teacher-forced logits of both forms are equally close to the oracle,
        # tools/diag_xattn_rows.py).  So a window that differs must be EPS-optimal under the oracle's beam search in
        # BOTH forms, every token rule-legal, as tests/test_gpu_decode.py requires of the default form.
        from oracle.decode import generate_one, score_sequence
        eps = {"tiny": 0.02, "base": 0.03, "small": 0.05}[dims.name]
        opt = GenerateOptions(beam_size=5, suppress_tokens=_sup(st), max_length=100)
        for w, (x, y) in enumerate(zip(ra, rb)):
            if x.tokens != y.tokens:
                cross = orc.cross_kv(encf[w: w + 1])
                r = generate_one(orc, cross, prompt, st, opt)
                for z in (x, y):
                    ended = len(prompt) + len(z.tokens) < 100
                    chosen, _, score = score_sequence(orc, cross, prompt, z.tokens, st, opt, ended)
                    assert np.all(np.isfinite(chosen)), (w, z.tokens)
                    assert score >= r.score - eps, (w, score, r.score)
        assert same >= W // 2, f"{same}/{W} windows identical"
    else:
        # greedy on random weights: a window may flip at a near-tied step (bf16 noise between the two forms);
        # then BOTH forms must be epsilon-consistent under the oracle, tie-aware (tests/parity_util.py)
        eps = {"tiny": 0.02, "base": 0.03, "small": 0.05}[dims.name]
        opt = GenerateOptions(beam_size=1, suppress_tokens=_sup(st), max_length=100)
        orc16 = OracleWhisper(orc.w, dims, np.float32, bf16_acts=True)     # the engine's numeric format
        for w, (x, y) in enumerate(zip(ra, rb)):
            if x.tokens != y.tokens:
                for r in (x, y):
                    wp = window_parity(orc16, encf[w], prompt, r, st, opt, w, eps=eps)
                    assert wp.min_margin_rule_tie >= -eps, (w, wp.min_margin_rule_tie, wp.worst_step)
        assert same >= W // 2, f"{same}/{W} windows identical"
    for x, y in zip(ra, rb):
        assert abs(x.no_speech_prob - y.no_speech_prob) < 2e-3
        if x.tokens == y.tokens:
            assert abs(x.score - y.score) < 2e-2 * max(1.0, abs(x.score))
    assert sum(len(r.tokens) for r in rb) > W * 5


def test_factored_prompted_prefill(small_models):
    """A long previous-text prompt: many rows per window (m-tiles > 1, fewer key splits)."""
    dims, eng, enc, orc, W = small_models
    st = dims.specials
    prompt = [st.sot_prev] + list(range(400, 500)) + [st.sot, st.lang_token("en"), st.transcribe]
    a, b = _both(eng, enc, W, 5 * W, lambda: eng.generate([0, 2], [prompt] * 2, beam_size=5, patience=1.0,
                                                            suppress_tokens=_sup(st), max_length=180)[0])
    assert sum(x.tokens == y.tokens for x, y in zip(a, b)) >= 1
    for x, y in zip(a, b):
        assert abs(x.no_speech_prob - y.no_speech_prob) < 2e-3


def test_large_v3_factored_matches_projected():
    """The bench instantiation (d = 1280: 8 waves x 160 columns), projected vs factored on the GPU."""
    W = 3
    dims, sd, eng, enc = _engine("large-v3", 1, W, eot_after=30)
    st = dims.specials
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe] + list(range(300, 330))])
    a, b = _both(eng, enc, W, 5 * W, lambda: eng.forward([2], toks)[0].cpu().numpy())
    assert np.abs(a - b).max() < 0.02 * max(np.abs(a).max(), 1.0), np.abs(a - b).max()
    prompt = [st.sot, st.lang_token("en"), st.transcribe]

    def run():
        return eng.generate(list(range(W)), [prompt] * W, suppress_tokens=_sup(st), max_length=80)[0]

    ra, rb = _both(eng, enc, W, 5 * W, run)
    # token identity between the two forms is decided by near-tied logits of the random model (their bf16
    # rounding differs): each form's tokens must be eps-consistent with the oracle (tie-aware teacher forcing)
    from oracle.decode import GenerateOptions
    from tests.parity_util import window_parity
    orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
    del sd
    encf = enc.float().cpu().numpy()
    opt = GenerateOptions(suppress_tokens=_sup(st), max_length=80)
    for res in (ra, rb):
        for w in range(W):
            r = window_parity(orc, encf[w], prompt, res[w], st, opt, w, eps=0.08)
            assert r.min_margin_rule_tie >= -0.08, (w, r)
            assert abs(r.no_speech_gpu - r.no_speech_oracle) < 1e-3
    assert sum(len(r.tokens) for r in rb) > W * 5
    eng.set_option("cross_mode", 1)
    assert eng.device_bytes() > 0


def test_large_v3_dma_form_bit_identical():
    """The LDS-DMA form of the factored attention (option cross_attn_dma, d = 1280) against the register-staged form
    (the default), both on key-split items (cross_attn_chunks 0): the same work items, per-wave MFMAs and
    fixed-order cross-wave sums, so the same bits -- teacher-forced logits over a 40-row prompt (two m-tiles per
    window), alignment-head capture on the attention kernel (cross_tf 0), greedy and beam-5 decodes (1 and 5 rows per
    window, rows finishing at different steps).  Then the stream-K chunk cut for greedy passes (opt-in): the
    register form (a chunk's segments as work items) and the LDS-DMA form (a workgroup walks its chunk) give the
    same bits; beam and teacher-forced passes are untouched (more than one m-tile per window: items); greedy agrees
    with the key-split cut to f32 rounding (a window's pieces differ from its key splits); and slicing a pass into
    two launches (decode_split: 32 greedy rows, two slices of 16) changes no bit."""
    W, WB = 32, 4                                     # greedy over 32 windows, beam over 4
    dims, sd, eng, enc = _engine("large-v3", 2, W, eot_after=30)
    del sd
    st = dims.specials
    heads = dims.default_alignment_heads()
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe, st.no_timestamps] + list(range(500 + 40 * i, 536 + 40 * i))
                     for i in range(2)])
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    assert eng.option("cross_attn_dma") == 0 and eng.option("cross_attn_chunks") == 0     # the defaults
    out = {}
    try:
        for form, chunks, split in ((0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0), (0, 1, 1)):
            eng.set_option("cross_attn_dma", form)
            eng.set_option("cross_attn_chunks", chunks)
            eng.set_option("decode_split", split)
            eng.set_option("cross_tf", 0)
            eng.reserve(W, 5 * W)
            eng.cross_kv(enc, 0)
            lg, at = eng.forward([3, 1], toks, align_heads=heads)
            eng.set_option("cross_tf", 1)
            one = eng.forward(list(range(W)), np.array([[st.sot]] * W))[0].cpu().numpy()   # one row per window
            g, _ = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=_sup(st), max_length=60)
            b, _ = eng.generate(list(range(WB)), [prompt] * WB, beam_size=5, patience=1.0, suppress_tokens=_sup(st),
                                max_length=60)
            out[(form, chunks, split)] = (lg.cpu().numpy(), at.cpu().numpy(), g, b, one)
    finally:
        eng.set_option("cross_attn_dma", 0)
        eng.set_option("cross_attn_chunks", 0)
        eng.set_option("decode_split", 0)
        eng.set_option("cross_tf", 1)

    def same(x, y, greedy=True):
        if greedy:
            assert np.array_equal(x[4], y[4]), np.abs(x[4] - y[4]).max()
        assert np.array_equal(x[0], y[0]), np.abs(x[0] - y[0]).max()
        assert np.array_equal(x[1], y[1]), np.abs(x[1] - y[1]).max()
        for ra, rb in (((x[2], y[2]),) if greedy else ()) + ((x[3], y[3]),):
            assert [r.tokens for r in ra] == [r.tokens for r in rb]
            assert [r.score for r in ra] == [r.score for r in rb]
            assert [r.no_speech_prob for r in ra] == [r.no_speech_prob for r in rb]

    reg, items, chunks, dchunks, sliced = (out[(0, 0, 0)], out[(1, 0, 0)], out[(0, 1, 0)], out[(1, 1, 0)],
                                           out[(0, 1, 1)])
    assert np.all(np.isfinite(items[0])) and np.allclose(items[1].sum(-1), 1.0, atol=1e-4)
    same(reg, items)                  # the two forms on key-split items
    same(chunks, dchunks)             # ... and on the chunk cut (register: segments as items; LDS-DMA: chunk walks)
    same(items, chunks, greedy=False)
    same(chunks, sliced)
    # the chunk cut vs the key splits on the same one-row-per-window pass: f32 rounding of the piece merge, then bf16
    # activations downstream
    diff = np.abs(items[4] - chunks[4]).max()
    assert diff < 0.01 * max(np.abs(items[4]).max(), 1.0), diff
    for x, y in zip(items[2], chunks[2]):
        assert abs(x.no_speech_prob - y.no_speech_prob) < 1e-3
        if x.tokens == y.tokens:
            assert abs(x.score - y.score) < 2e-3 * max(1.0, abs(x.score)), (x.score, y.score)
    # random weights: near-tied greedy steps part on rounding noise (test_large_v3_factored_matches_projected); the
    # records sweeps (test_gpu_logprobs, test_gpu_configs) hold the default cut to the oracle
    assert sum(x.tokens == y.tokens for x, y in zip(items[2], chunks[2])) >= W // 2
    assert sum(len(r.tokens) for r in chunks[2]) > W * 5
