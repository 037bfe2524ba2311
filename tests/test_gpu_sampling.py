"""Sampling and the temperature-fallback policy (faster-whisper generate_with_fallback, BASELINE A8) vs the oracle.

The engine samples by Gumbel-max with counter-based noise keyed on (call seed, hypothesis row, step, token)
(vlog_amd/csrc/search.hip `gumbel`), restated bit for bit in oracle/decode.py `gumbel_noise`; so at T > 0 the
oracle reproduces the GPU's draws and the check is the same as at T = 0: identical hypotheses, or every GPU
token within eps of the oracle's best Gumbel key at its step (bf16 logit noise at a near-tie of the keys).
"""
import numpy as np
import pytest
import torch

from oracle import mel as omel
from oracle import transcribe as otr
from oracle.decode import GenerateOptions, apply_rules, generate_one, gumbel_noise
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu
EPS = 0.02          # nats: bf16 logit noise at a near-tie of two Gumbel keys
RULE_EPS = 0.05     # the timestamp-forcing gap is a difference of two log-sum-exps: its noise is larger


@pytest.fixture(scope="module")
def setup():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=3, eot_after=60)
    eng = GpuEngine(dims, sd, 0)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
    W = 4
    x = np.concatenate([speech_like(30.0, 800 + i) for i in range(W)])
    feats = omel.log_mel(x, dims.n_mels)
    enc = eng.encode(torch.from_numpy(feats).cuda(), [3000 * i for i in range(W)], [3000] * W)
    eng.reserve(W, 16)
    eng.cross_kv(enc, 0)
    return dims, eng, orc, enc.float().cpu().numpy(), W


def _key_margins(orc, cross, prompt, tokens, st, opt, hyp, ended):
    """Teacher-force `tokens` (a GPU sample) with the engine's Gumbel noise of hypothesis `hyp`: per step, the
    chosen token's key minus the best key — on the other side of the timestamp-forcing rule too when the oracle
    takes that decision within EPS of its threshold (a hard threshold on logits: tests/parity_util.py)."""
    from oracle.decode import log_softmax
    seq = list(tokens) + ([st.eot] if ended else [])
    logits, _ = orc.decode(np.asarray([list(prompt) + list(tokens)]), cross)
    P = len(prompt)
    tb = st.timestamp_begin
    out = []
    for i, t in enumerate(seq):
        row, hist = logits[0, P - 1 + i], list(tokens[:i])
        g = gumbel_noise(opt.seed, hyp, i, row.shape[0])
        xp = apply_rules(row, hist, st, opt.suppress_tokens, opt.suppress_blank, opt.max_initial_timestamp_index,
                         opt.with_timestamps, force_timestamps=False)
        lpp = log_softmax(xp)
        text_max = float(np.max(lpp[:tb]))
        gap = float(np.logaddexp.reduce(lpp[tb:]) - text_max) if np.isfinite(text_max) else -np.inf
        branches = [gap > 0] + ([gap <= 0] if abs(gap) <= RULE_EPS else [])
        best = -np.inf
        for forced in branches:
            x = xp.copy()
            if forced:
                x[:tb] = -np.inf
            k = x / opt.sampling_temperature + g
            best = max(best, float(k[t] - np.max(k)))
        out.append((best, gap))
    return np.array(out)


def test_gumbel_noise_restatement_properties():
    g = gumbel_noise(5, 3, 7, 200000)
    assert np.all(np.isfinite(g))
    assert g.dtype == np.float32 and abs(float(g.mean()) - 0.5772) < 0.01 and abs(float(g.std()) - 1.2825) < 0.01
    assert np.array_equal(g, gumbel_noise(5, 3, 7, 200000)) and not np.array_equal(g, gumbel_noise(5, 4, 7, 200000))


@pytest.mark.parametrize("T", [0.4, 1.0])
def test_sampling_matches_oracle_draws(setup, T):
    dims, eng, orc, encf, W = setup
    st = dims.specials
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    sup = [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]
    nh, seed = 3, 11
    res, _ = eng.generate(list(range(W)), [prompt] * W, temperature=T, num_hypotheses=nh, seed=seed,
                          suppress_tokens=sup, max_length=120)
    same = 0
    for w in range(W):
        cross = orc.cross_kv(encf[w: w + 1])
        opt = GenerateOptions(suppress_tokens=sup, max_length=120, sampling_temperature=T, num_hypotheses=nh,
                              seed=seed, hyp_offset=w * nh)
        r = generate_one(orc, cross, prompt, st, opt)
        same += r.tokens == res[w].tokens
        ended = len(prompt) + len(res[w].tokens) < 120
        # the GPU's pick came from one of the window's nh hypotheses: eps-consistent under that one's noise
        per_j = [_key_margins(orc, cross, prompt, res[w].tokens, st, opt, w * nh + j, ended) for j in range(nh)]
        j = int(np.argmax([m[:, 0].min() for m in per_j]))
        k = int(np.argmin(per_j[j][:, 0]))
        assert per_j[j][k, 0] >= -EPS, (w, j, k, per_j[j][k].tolist(), len(res[w].tokens))
        assert abs(r.no_speech_prob - res[w].no_speech_prob) < 1e-3
    assert same >= W // 2, same          # a near-tied key or forcing decision diverges the rest of a sample


@pytest.mark.parametrize("mfma", [1, 0])
def test_sampling_projected_rows_end_apart(setup, mfma):
    """best_of sampling in the PROJECTED cross form (cross_mode 0: what transcribe.py runs for beam / best-of groups)
    with the MFMA group kernel (cross_mfma 1) and the VALU one (0).  A window's 5 sampled hypotheses end at different
    steps; every live row must keep its cross-attention after another row of its group has ended (the MFMA kernel
    once returned for the whole group when its first row was done).  Checked per step: the chosen
    hypothesis' log-prob records vs the oracle teacher-forced on the same tokens (0.02 nats), and each token within
    eps of the oracle's best Gumbel key under that hypothesis' noise."""
    from tests.parity_util import oracle_records, record_deviation
    dims, eng, orc, encf, W = setup
    st = dims.specials
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    sup = [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]
    nh, seed, T, ML = 5, 23, 0.4, 120
    eng.set_option("cross_mode", 0)
    eng.set_option("cross_mfma", mfma)
    try:
        eng.reserve(W, W * nh)
        eng.cross_kv(torch.from_numpy(encf).to(torch.bfloat16).cuda(), 0)
        res, _ = eng.generate(list(range(W)), [prompt] * W, temperature=T, num_hypotheses=nh, seed=seed,
                              suppress_tokens=sup, max_length=ML, record_logprobs=True)
    finally:
        eng.set_option("cross_mode", 1)
        eng.set_option("cross_mfma", 1)
        eng.cross_kv(torch.from_numpy(encf).to(torch.bfloat16).cuda(), 0)
    lens = [len(r.tokens) for r in res]
    assert len(set(lens)) > 1, lens
    opt = GenerateOptions(suppress_tokens=sup, max_length=ML, sampling_temperature=T, num_hypotheses=nh, seed=seed)
    worst = 0.0
    for w in range(W):
        rec = oracle_records(orc, encf[w: w + 1], prompt, [res[w].tokens], 1, st, opt)[0]
        dev, _ = record_deviation(res[w].token_logprobs, rec)
        worst = max(worst, float(dev.max()))
        cross = orc.cross_kv(encf[w: w + 1])
        ended = len(prompt) + len(res[w].tokens) < ML
        o = GenerateOptions(suppress_tokens=sup, max_length=ML, sampling_temperature=T, num_hypotheses=nh,
                            seed=seed, hyp_offset=w * nh)
        per_j = [_key_margins(orc, cross, prompt, res[w].tokens, st, o, w * nh + j, ended) for j in range(nh)]
        assert max(m[:, 0].min() for m in per_j) >= -EPS, (w, lens)
    assert worst <= 0.02, worst


class _GpuBackend:
    def __init__(self, m):
        self.m = m

    def encode(self, window):
        enc = self.m.engine.encode(torch.from_numpy(np.ascontiguousarray(window, dtype=np.float32)).cuda(), [0], [3000])
        self.m.engine.cross_kv(enc, 0)
        return 0

    def generate(self, slot, prompt, opt):
        from oracle.decode import GenerateResult
        st = self.m.dims.specials
        res, _ = self.m.engine.generate([slot], [prompt], beam_size=opt.beam_size, patience=opt.patience,
                                        length_penalty=opt.length_penalty, max_length=opt.max_length,
                                        temperature=opt.sampling_temperature, num_hypotheses=opt.num_hypotheses,
                                        seed=opt.seed, suppress_tokens=opt.suppress_tokens,
                                        suppress_blank=opt.suppress_blank,
                                        max_initial_timestamp_index=opt.max_initial_timestamp_index,
                                        sot_index=prompt.index(st.sot))
        r = res[0]
        return GenerateResult(r.tokens, r.score, r.no_speech_prob, r.cum_logprob)

    def detect_language(self, slot):
        raise AssertionError("language is given")


class _Dims:
    def __init__(self, dims):
        self.dims = dims


def test_fallback_policy_matches_oracle_host_loop():
    """Default temperatures (0, 0.2, ..., 1.0), beam 5: the random model fails the log-prob threshold, so every
    window walks the whole fallback ladder with best_of 5 sampling.  The product's generate_with_fallback +
    seek loop vs oracle/transcribe.py on the same GPU decoder: identical segments, accepted temperature,
    avg_logprob and compression ratio."""
    from vlog_amd.transcribe import WhisperModel
    model = WhisperModel("synthetic:tiny:3", device="cuda", eot_after=60)
    x = np.concatenate([speech_like(30.0, 810), speech_like(21.0, 811)])
    segs, info = model.transcribe(x, language="en", beam_size=5)
    segs = list(segs)
    assert segs
    feats = model.engine.features(torch.from_numpy(x)).cpu().numpy()
    ref, _ = otr.transcribe(_Dims(model.dims), lambda l: Tokenizer(model.dims, language=l), x, beam_size=5,
                            language="en", features=feats, backend=_GpuBackend(model))
    assert [s.tokens for s in segs] == [r["tokens"] for r in ref]
    for s, r in zip(segs, ref):
        assert s.temperature == r["temperature"]
        assert abs(s.avg_logprob - r["avg_logprob"]) < 1e-9
        assert (s.start, s.end) == (r["start"], r["end"])
