"""Per-step log-prob parity of the exact kernels the bench times, on RANDOM-init weights.

The margin-planted gates (tests/test_gpu_gates.py) decide every token by tens to thousands of nats, so they cannot
fail on arithmetic.  Here the engine records, at every generated step of every window, the log-prob (after the
logit rules) of the token it chose and of the best other allowed token (wm_generate h_token_logprobs /
h_token_logprobs_other; search.hip).  Every window's tokens are teacher-forced through the CPU oracle in the
engine's numeric format (bf16 activations, oracle/model.py bf16_acts) from the GPU's own encoder output, and the
oracle's log-prob of the same token at the same step must agree with the GPU's record:

    |lp_gpu - lp_oracle| <= BAR = 0.02 nats at EVERY step of EVERY window

(the bar tests/test_gpu_parity.py:95 holds for raw logits on tiny).  Where the oracle's own timestamp-forcing
decision sits within 0.05 nats of its threshold (the rule is a hard threshold on logits), the record may sit on the
other side (parity_util.record_deviation); such steps are counted and reported.

Configs (BASELINE.json): 2 base greedy 32 windows, 3 small greedy 120 windows, 4 large-v3 greedy 150 windows
(the bench's decode: 150 rows through dec_ring / xattn<160> / logits_select), 5 large-v3 beam 5 over 128
windows (640 rows, projected cross form as the product runs beam groups), and the opt-in fp8 cross memory against
the FULL-precision oracle (its accuracy cost, bounded by FP8_BAR / FP8_P99).  Reference call:
worker/transcription.py:105-131.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.decode import GenerateOptions
from oracle.model import OracleWhisper
from tests.parity_util import oracle_records, progress, record_deviation, source_offset
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu

BAR = 0.02          # nats, bf16 engine vs bf16-format oracle, every step
FP8_BAR = 0.05      # nats, fp8 cross memory vs the full-precision oracle, every step (max; measured 0.014)
FP8_P99 = 0.02      # nats, its 99th percentile over all steps (measured 0.0087)
# large-v3: every step of every STRIDE-th window of the batch (windows OFFSET, OFFSET + STRIDE, ...) goes through the
# oracle (the whole batch decodes on the GPU either way); VLOG_AMD_RECORDS_STRIDE=1 sweeps every window
# (profiles/parity_r4_a_records_failure.jsonl)
STRIDE = max(1, int(os.environ.get("VLOG_AMD_RECORDS_STRIDE", "4")))


OFFSET = source_offset(STRIDE, "VLOG_AMD_RECORDS_OFFSET")


def _record(name, **kw):
    p = os.environ.get("VLOG_AMD_PARITY_OUT")
    if p:
        with open(p, "a") as f:
            f.write(json.dumps(dict(name=name, **kw)) + "\n")


class RandomConfig:
    def __init__(self, name, n_windows, eot_after=110, seed=0):
        from vlog_amd.engine import GpuEngine
        self.dims = dims = model_dims(name)
        sd = synthetic_state_dict(dims, seed=seed, eot_after=eot_after)
        self.eng = GpuEngine(dims, sd, 0)
        self.orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
        del sd
        self.W = n_windows
        x = np.concatenate([speech_like(30.0, i) for i in range(n_windows)])
        self.mel = self.eng.features(torch.from_numpy(x))
        self.enc = self.eng.encode(self.mel, [3000 * i for i in range(n_windows)], [3000] * n_windows)
        self.tok = Tokenizer(dims, language="en")
        self.prompt = list(self.tok.sot_sequence)
        self.sup = list(self.tok.suppressed_tokens([-1]))
        self.st = dims.specials

    def opt(self, beam=1):
        return GenerateOptions(beam_size=beam, suppress_tokens=self.sup, max_length=448)

    def generate(self, W=None, **kw):
        W = self.W if W is None else W
        self.eng.reserve(self.W, W * kw.get("beam_size", 1))
        self.eng.cross_kv(self.enc, 0)
        res, _ = self.eng.generate(list(range(W)), [self.prompt] * W, suppress_tokens=self.sup, max_length=448,
                                   check_every=4, record_logprobs=True, **kw)
        return res

    def enc_of(self, ws):
        return self.enc[list(ws)].float().cpu().numpy()


def sweep(cfg: RandomConfig, runs, chunk=8, stride=1, offset=0):
    """runs: {name: list of GenResult by window (None past its windows)}.  Every `stride`-th window's sequences of
    every run (from window `offset`) teacher-forced through the oracle together (one cross-KV per window), per-step
    deviations per run."""
    names = list(runs)
    W = max(len(r) for r in runs.values())
    sel = list(range(offset % stride, W, stride))
    dev = {n: [] for n in names}
    ties = {n: 0 for n in names}
    worst = {n: (0.0, -1, -1) for n in names}
    margin = {n: 0.0 for n in names}
    for c0 in range(0, len(sel), chunk):
        progress(f"logprob sweep {cfg.dims.name}: windows {c0}/{len(sel)}")
        ws = sel[c0: c0 + chunk]
        seqs, who = [], []
        for w in ws:
            for n in names:
                r = runs[n][w] if w < len(runs[n]) else None
                seqs.append(list(r.tokens) if r is not None else [])
                who.append((n, w, r))
        rep = len(names)
        recs = oracle_records(cfg.orc, cfg.enc_of(ws), cfg.prompt, seqs, rep, cfg.st, cfg.opt())
        for (n, w, r), rec in zip(who, recs):
            if r is None:
                continue
            d, t = record_deviation(r.token_logprobs, rec)
            dev[n].append(d)
            # the oracle's margin of the GPU's token over the best other (tie-aware as record_deviation): a greedy
            # decode must have picked the oracle's best to within the noise bar
            tie = (np.abs(rec[:, 2]) <= 0.05) & (np.abs(np.asarray(r.token_logprobs) - rec[:, 1]) < d + 1e-12)
            margin[n] = min(margin[n], float(np.min(np.where(tie, 0.0, rec[:, 0] - rec[:, 3]))) if len(rec) else 0.0)
            ties[n] += t
            k = int(np.argmax(d)) if d.size else -1
            if d.size and d[k] > worst[n][0]:
                worst[n] = (float(d[k]), w, k)
        del recs
    out = {}
    for n in names:
        a = np.concatenate(dev[n]) if dev[n] else np.zeros(0)
        out[n] = dict(steps=int(a.size), max=float(a.max()) if a.size else 0.0,
                      p99=float(np.percentile(a, 99)) if a.size else 0.0, mean=float(a.mean()) if a.size else 0.0,
                      over_bar=int((a > BAR).sum()), rule_tie_steps=ties[n], worst=worst[n],
                      min_oracle_margin=margin[n])
    return out


def _self_consistent(res):
    """The records sum to the engine's own cumulative log-prob (every step recorded exactly once)."""
    for r in res:
        assert r.token_logprobs is not None and np.isfinite(r.token_logprobs).all()
        assert abs(float(np.sum(r.token_logprobs, dtype=np.float64)) - r.cum_logprob) < 1e-3 * max(1.0, abs(r.cum_logprob))


def _greedy_case(name, W):
    cfg = RandomConfig(name, W)
    res = cfg.generate()
    _self_consistent(res)
    s = sweep(cfg, {"greedy": res})["greedy"]
    _record(f"logprob records {name} greedy {W} windows", bar=BAR, **s)
    assert s["max"] <= BAR and s["min_oracle_margin"] >= -BAR, s
    return cfg, res


def test_config2_base_32_windows_every_step():
    _greedy_case("base", 32)


def test_config3_small_120_windows_every_step():
    _greedy_case("small", 120)


def test_row_set_decode_every_step():
    """The row-set decode (max_rows < windows: refills inside the decoder pass, then compaction) on config 2's
    windows: the same per-step bar, and its tokens those of the all-rows decode wherever the two agree to
    within BAR at every step (routes differ with the pass's row count: f32 rounding, not bit for bit)."""
    cfg = RandomConfig("base", 32)
    ref = cfg.generate()
    st = {}
    res = cfg.generate(max_rows=12, compact=True, stats=st)
    assert st["refills"] == 32 - 12 and st["passes"] > 0, st
    _self_consistent(res)
    s = sweep(cfg, {"rows": res})["rows"]
    same = sum(a.tokens == b.tokens for a, b in zip(ref, res))
    _record("logprob records base greedy 32 windows, row-set decode (12 rows, compact)", bar=BAR, same_tokens=same,
            stats=st, **s)
    assert s["max"] <= BAR, s
    # the random model's near-ties part the two decodes on some windows (22/32 identical measured); every token of
    # the row-set decode is the oracle's greedy choice to within the bar
    assert s["min_oracle_margin"] >= -BAR, s


@pytest.fixture(scope="module")
def lv3():
    return RandomConfig("large-v3", 150)


def test_config4_5_large_v3_greedy_beam_fp8_every_step(lv3):
    """Config 4 (150 windows greedy, the bench's kernels), config 5's search (beam 5 over 128 windows, the
    projected form the product uses for beam groups) and the opt-in fp8 cross memory (vs the full-precision
    oracle) in one oracle sweep (one cross-KV per window for the three runs; every STRIDE-th window)."""
    greedy = lv3.generate()
    _self_consistent(greedy)
    lv3.eng.set_option("cross_fp8", 1)
    try:
        fp8 = lv3.generate()
    finally:
        lv3.eng.set_option("cross_fp8", 0)
    lv3.eng.set_option("cross_mode", 0)
    try:
        beam = lv3.generate(W=128, beam_size=5, patience=1.0)
    finally:
        lv3.eng.set_option("cross_mode", 1)
    for r in beam:
        assert r.token_logprobs is not None and np.isfinite(r.token_logprobs).all()
        assert abs(float(np.sum(r.token_logprobs, dtype=np.float64)) - r.cum_logprob) < 1e-3 * max(1.0, abs(r.cum_logprob))
    s = sweep(lv3, {"greedy": greedy, "fp8": fp8, "beam5": beam}, stride=STRIDE, offset=OFFSET)
    same_fp8 = sum(a.tokens == b.tokens for a, b in zip(greedy, fp8))
    _record(f"logprob records large-v3: greedy 150 / fp8 150 (vs full-precision oracle) / beam5 128, every step of "
            f"every {STRIDE}th window", bar=BAR, fp8_bar=FP8_BAR, fp8_p99_bar=FP8_P99, stride=STRIDE, offset=OFFSET,
            fp8_windows_identical_to_bf16=same_fp8, **s)
    assert s["greedy"]["max"] <= BAR and s["greedy"]["min_oracle_margin"] >= -BAR, s["greedy"]
    assert s["beam5"]["max"] <= BAR, s["beam5"]
    assert s["fp8"]["max"] <= FP8_BAR and s["fp8"]["p99"] <= FP8_P99, s["fp8"]


def test_large_v3_ln_fold_opt_in_every_step(lv3):
    """The opt-in folded LayerNorm decode (decode_ln_fold=1: the residual producer writes bf16(x * gamma) and row
    sums, the consumer GEMM's epilogue applies the LayerNorm; measured slower than the default, kept for A/B) on 48
    large-v3 windows (ring passes): the same per-step bar against the oracle."""
    lv3.eng.set_option("decode_ln_fold", 1)
    try:
        res = lv3.generate(W=48)
    finally:
        lv3.eng.set_option("decode_ln_fold", 0)
    _self_consistent(res)
    s = sweep(lv3, {"fold": res}, stride=STRIDE, offset=OFFSET)["fold"]
    _record(f"logprob records large-v3 greedy 48 windows, decode_ln_fold=1, every {STRIDE}th window", bar=BAR,
            stride=STRIDE, offset=OFFSET, **s)
    assert s["max"] <= BAR and s["min_oracle_margin"] >= -BAR, s
