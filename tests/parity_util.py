"""Generate-boundary parity helpers shared by the GPU tests and bench.py's parity sample (test infrastructure:
imports oracle/ as the checker only).

`teacher_force` runs the GPU's generated tokens through the CPU oracle in ONE batched decoder pass (prompt +
tokens) and applies the same logit rules at every step.  If the GPU's token is the oracle's argmax at every
step, the oracle's own greedy search would have produced exactly the same sequence (induction on the step),
so "identical" below is token identity with the oracle's greedy decode, at the cost of one forward pass
instead of one pass per token.
"""
from __future__ import annotations

import json
import os
import sys
from dataclasses import asdict, dataclass
from typing import List, Optional, Sequence

import numpy as np

from oracle.decode import GenerateOptions, apply_rules, log_softmax


@dataclass
class WindowParity:
    window: int
    n_tokens: int
    identical: bool            # GPU token == oracle argmax at every step (=> oracle greedy == GPU tokens)
    min_margin: float          # min over steps of (logprob of the GPU token - best logprob), <= 0
    score_gpu: float
    score_oracle: float
    no_speech_gpu: float
    no_speech_oracle: float
    # epsilon-consistency that also accepts the other side of a rule threshold the oracle itself sits within
    # eps of (see teacher_force): min over steps of max(margin, margin on the other side when |gap| <= eps)
    min_margin_rule_tie: float = 0.0
    worst_step: int = -1
    worst_gap: float = 0.0     # the timestamp-forcing gap (log P(timestamp) - max text logprob) at that step


def rule_margins(logits_row, sampled, st, opt: GenerateOptions, token: int):
    """Margin of `token` under the oracle's rules, plus the timestamp-forcing gap and the margin on the other
    side of that rule.  faster-whisper / CTranslate2's ApplyTimestampRules forces a timestamp when the
    timestamp tokens' total probability exceeds the best text token's; that decision is a hard threshold on
    logits, so a bf16 logit difference far below the noise floor can flip it when the two sides are nearly
    equal (observed on the random-weight models, whose timestamp mass sits near the best text token)."""
    x = apply_rules(logits_row, sampled, st, opt.suppress_tokens, opt.suppress_blank, opt.max_initial_timestamp_index,
                    opt.with_timestamps)
    lp = log_softmax(x)
    margin = float(lp[token] - np.max(lp))
    gap, alt, lp_alt = 0.0, margin, float(lp[token])
    if opt.with_timestamps:
        tb = st.timestamp_begin
        # rebuild the pre-forcing logits: apply_rules without the final forcing step
        xp = apply_rules(logits_row, sampled, st, opt.suppress_tokens, opt.suppress_blank,
                         opt.max_initial_timestamp_index, opt.with_timestamps, force_timestamps=False)
        lpp = log_softmax(xp)
        text_max = float(np.max(lpp[:tb]))
        if np.isfinite(text_max):
            gap = float(np.logaddexp.reduce(lpp[tb:]) - text_max)
            forced = gap > 0
            xo = xp.copy()
            if not forced:
                xo[:tb] = -np.inf                      # the other side of the threshold
            lpo = log_softmax(xo)
            alt = float(lpo[token] - np.max(lpo)) if np.isfinite(lpo[token]) else -np.inf
            lp_alt = float(lpo[token])
    return margin, gap, alt, float(lp[token]), lp_alt


def teacher_force(orc, cross, prompt: Sequence[int], tokens: Sequence[int], st, opt: GenerateOptions,
                  ended_with_eot: bool):
    """-> (chosen logprobs, best logprobs, normalised score, no_speech_prob) of `tokens` under the oracle."""
    seq = list(tokens) + ([st.eot] if ended_with_eot else [])
    toks = np.asarray([list(prompt) + list(tokens)])
    logits, _ = orc.decode(toks, cross)
    P = len(prompt)
    chosen, best = [], []
    for i, t in enumerate(seq):
        x = apply_rules(logits[0, P - 1 + i], list(tokens[:i]), st, opt.suppress_tokens, opt.suppress_blank,
                        opt.max_initial_timestamp_index, opt.with_timestamps)
        lp = log_softmax(x)
        chosen.append(float(lp[t]))
        best.append(float(np.max(lp)))
    ns = 0.0
    if st.sot in prompt:
        p = np.exp(log_softmax(logits[0, list(prompt).index(st.sot)]))
        ns = float(p[st.no_speech])
    score = float(np.sum(chosen)) / (max(len(tokens), 1) ** opt.length_penalty)
    return np.array(chosen), np.array(best), score, ns


def window_parity(orc, enc_window: np.ndarray, prompt, res, st, opt: GenerateOptions, window: int,
                  eps: float = 0.05) -> WindowParity:
    """res: vlog_amd.engine.GenResult of that window; enc_window [1500, d] float32 (the GPU's encoder output)."""
    cross = orc.cross_kv(enc_window[None])
    ended = len(prompt) + len(res.tokens) < opt.max_length
    tokens = list(res.tokens)
    seq = tokens + ([st.eot] if ended else [])
    logits, _ = orc.decode(np.asarray([list(prompt) + tokens]), cross)
    P = len(prompt)
    margins, tie_margins, gaps = [], [], []
    cum = 0.0
    for i, t in enumerate(seq):
        row = logits[0, P - 1 + i]
        m, gap, alt, lp_t, lp_alt = rule_margins(row, tokens[:i], st, opt, t)
        tie = abs(gap) <= eps and alt > m              # the GPU took the other side of a near-tied rule
        cum += lp_alt if tie else lp_t
        margins.append(m)
        gaps.append(gap)
        tie_margins.append(alt if tie else m)
    ns = 0.0
    if st.sot in prompt:
        ns = float(np.exp(log_softmax(logits[0, list(prompt).index(st.sot)]))[st.no_speech])
    score = cum / (max(len(tokens), 1) ** opt.length_penalty)
    margins = np.array(margins)
    # fully masked rows are -inf (oracle.decode.log_softmax), never NaN: a NaN here is a checker bug, and
    # Python's min() would silently skip it
    assert not np.isnan(margins).any() and not np.isnan(np.asarray(tie_margins, dtype=np.float64)).any(), margins
    k = int(np.argmin(tie_margins)) if tie_margins else -1
    return WindowParity(window, len(tokens), bool(np.all(margins >= 0.0)), float(margins.min()) if margins.size else 0.0,
                        float(res.score), score, float(res.no_speech_prob), ns,
                        float(min(tie_margins)) if tie_margins else 0.0, k, float(gaps[k]) if k >= 0 else 0.0)


def record(name: str, rows: List[WindowParity], **extra) -> dict:
    """Summary dict; also appended as one JSON line to $VLOG_AMD_PARITY_OUT when that is set."""
    out = {"name": name, "n": len(rows), "identical": int(sum(r.identical for r in rows)),
           "min_margin": min((r.min_margin for r in rows), default=0.0),
           "min_margin_rule_tie": min((r.min_margin_rule_tie for r in rows), default=0.0),
           "max_score_diff": max((abs(r.score_gpu - r.score_oracle) for r in rows), default=0.0),
           "max_no_speech_diff": max((abs(r.no_speech_gpu - r.no_speech_oracle) for r in rows), default=0.0),
           "windows": [asdict(r) for r in rows]}
    out.update(extra)
    path = os.environ.get("VLOG_AMD_PARITY_OUT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(out) + "\n")
    return out


def source_offset(stride: int, env: str) -> int:
    """Which residue class of windows a strided sweep covers.  Deterministic by default (0), so the gated subset does
    not move between commits that never touched it.  The environment variable `env` pins another class;
    `VLOG_AMD_SWEEP_ROTATE=1` seeds it from the tree's kernel sources instead (the separate, recorded rotating sweep:
    every change of the HIP code then covers other windows).  Tests record the offset with their results."""
    if env in os.environ:
        return int(os.environ[env]) % stride
    if os.environ.get("VLOG_AMD_SWEEP_ROTATE") != "1":
        return 0
    import glob
    import hashlib
    h = hashlib.sha256()
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vlog_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(root, "*.hip")) + glob.glob(os.path.join(root, "*.cpp"))):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return int.from_bytes(h.digest()[:4], "little") % stride


def sample_indices(n: int, k: int) -> List[int]:
    """k window indices spread over [0, n), first and last included."""
    if k >= n:
        return list(range(n))
    return sorted({int(round(i * (n - 1) / (k - 1))) for i in range(k)})


# ------------------------------------------------------------------------------------------------ north_star gates
GATE_IDENTICAL = 0.99      # greedy token sequences identical on >= 99 % of windows
GATE_WER = 0.003           # WER delta <= 0.3 % absolute
GATE_DT = 0.02             # segment start / end within one timestamp token (20 ms)


def progress(msg: str) -> None:
    """One line to the terminal past pytest's capture, and to $VLOG_AMD_PROGRESS when set (long oracle checks on the
    GPU box keep their output moving: a runner that watches for silence must not take them for a hang)."""
    cf = sys.modules.get("vlog_amd_test_conftest")
    if cf is not None:
        try:
            cf.terminal_line(msg)
        except Exception:
            pass
    path = os.environ.get("VLOG_AMD_PROGRESS")
    if path:
        with open(path, "a") as f:
            f.write(msg + "\n")


def teacher_force_batch(orc, enc: np.ndarray, prompt: Sequence[int], token_lists: Sequence[Sequence[int]],
                        ended: Sequence[bool], st, opt: GenerateOptions):
    """Several windows in ONE oracle decoder pass (sequences padded with <|endoftext|>: the mask is causal, so
    padding never changes an earlier position).  -> per window: (margins [steps], no_speech_prob, cum_logprob) with
    margin = logprob of the GPU token minus the best logprob among the OTHER tokens (> 0: the oracle's argmax) and
    cum_logprob = the oracle's summed log-prob (after the rules) of the GPU tokens incl. the final <|endoftext|>."""
    cross = orc.cross_kv(enc)
    L = max(len(t) for t in token_lists)
    toks = np.full((len(token_lists), len(prompt) + L), st.eot, dtype=np.int64)
    for i, t in enumerate(token_lists):
        toks[i, :len(prompt)] = prompt
        toks[i, len(prompt):len(prompt) + len(t)] = t
    logits, _ = orc.decode(toks, cross)
    P = len(prompt)
    out = []
    for i, t in enumerate(token_lists):
        seq = list(t) + ([st.eot] if ended[i] else [])
        ms = np.empty(len(seq))
        cum = 0.0
        for k, tok in enumerate(seq):
            # the margin of the rule-masked logits equals that of their log-softmax (same shift)
            x = apply_rules(logits[i, P - 1 + k], list(t[:k]), st, opt.suppress_tokens, opt.suppress_blank,
                            opt.max_initial_timestamp_index, opt.with_timestamps)
            cum += float(log_softmax(x)[tok])
            chosen = x[tok]
            x[tok] = -np.inf
            ms[k] = chosen - np.max(x) if np.isfinite(chosen) else -np.inf
        assert not np.isnan(ms).any()
        ns = 0.0
        if st.sot in prompt:
            ns = float(np.exp(log_softmax(logits[i, list(prompt).index(st.sot)]))[st.no_speech])
        out.append((ms, ns, cum))
    return out


def step_logprobs(x_row: np.ndarray, sampled: Sequence[int], tok: int, st, opt: GenerateOptions):
    """The oracle's per-step record for the token `tok` chosen after `sampled`: (log-prob under the rules, log-prob
    on the other side of the timestamp-forcing threshold, the forcing gap log P(timestamps) - max log P(text),
    best log-prob among the other allowed tokens).  Restates search.hip's records (lp = logit - logsumexp of the
    allowed set) on the oracle's logits row."""
    xp = apply_rules(x_row, sampled, st, opt.suppress_tokens, opt.suppress_blank, opt.max_initial_timestamp_index,
                     opt.with_timestamps, force_timestamps=False)
    lpp = log_softmax(xp)
    tb = st.timestamp_begin
    gap, forced = 0.0, False
    xo = xp
    if opt.with_timestamps:
        text_max = float(np.max(lpp[:tb]))
        ts = float(np.logaddexp.reduce(lpp[tb:]))
        if np.isfinite(text_max) and np.isfinite(ts):
            gap = ts - text_max
        forced = ts > text_max
        xo = xp.copy()
        xo[:tb] = -np.inf                       # the forced form
    lpo = log_softmax(xo)
    lp_on, lp_off = (lpo, lpp) if forced else (lpp, lpo)
    other = lp_on.copy()
    other[tok] = -np.inf
    return float(lp_on[tok]), float(lp_off[tok]), gap, float(np.max(other))


def oracle_records(orc, enc: np.ndarray, prompt: Sequence[int], seqs: Sequence[Sequence[int]], rep: int, st,
                   opt: GenerateOptions):
    """Teacher-force `seqs` (window-major groups of `rep` sequences per window of `enc`) through the oracle in ONE
    decoder pass and return, per sequence, arrays (lp, lp_other_side_of_forcing, gap, best_other) over its steps
    (the generated tokens plus the final <|endoftext|> when the sequence ended before max_length)."""
    cross = orc.cross_kv(enc)
    P = len(prompt)
    L = max(1, max(len(s) for s in seqs))
    toks = np.full((len(seqs), P + L), st.eot, dtype=np.int64)
    for i, s in enumerate(seqs):
        toks[i, :P] = prompt
        toks[i, P:P + len(s)] = s
    logits, _ = orc.decode(toks, cross)

    def one(i):
        s = seqs[i]
        steps = list(s) + ([st.eot] if P + len(s) < opt.max_length else [])
        return np.array([step_logprobs(logits[i, P - 1 + k], list(s[:k]), t, st, opt) for k, t in enumerate(steps)],
                        dtype=np.float64).reshape(-1, 4)

    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=8) as pool:        # numpy's row ops release the GIL
        return list(pool.map(one, range(len(seqs))))


def record_deviation(gpu_lp: np.ndarray, rec: np.ndarray, eps_tie: float = 0.05):
    """|GPU record - oracle record| per step; at a step whose forcing gap the oracle itself sits within eps_tie of
    (the threshold decision is then ill-conditioned at bf16 noise), the other side of the threshold also counts.
    -> (deviation per step, number of tie steps where the other side was closer)."""
    g = np.asarray(gpu_lp, dtype=np.float64)
    assert g.shape[0] == rec.shape[0], (g.shape, rec.shape)
    dev = np.abs(g - rec[:, 0])
    tie = (np.abs(rec[:, 2]) <= eps_tie) & (np.abs(g - rec[:, 1]) < dev)
    dev = np.where(tie, np.abs(g - rec[:, 1]), dev)
    assert not np.isnan(dev).any(), "NaN in a per-step record"
    return dev, int(tie.sum())


def gate_windows(orc, enc_of, prompt: Sequence[int], results, st, opt: GenerateOptions, tokenizer,
                 windows: Optional[Sequence[int]] = None, chunk: int = 8, time_offset=lambda w: 0.0,
                 known: Optional[dict] = None) -> dict:
    """The north_star parity gates over every window (or `windows`): each GPU token sequence is teacher-forced
    through the oracle (identical = the GPU token is the oracle's argmax at every step, so the oracle's greedy
    search produces exactly that sequence); windows that are not identical are re-decoded by the oracle's own
    greedy search.  WER delta = WER of the GPU transcript against the oracle transcript (per-window edit
    distances summed); segment times compared segment by segment (start/end within 20 ms).
    enc_of(list of window ids) -> float32 [n, 1500, d] (the GPU's encoder output: parity at the decoder).
    known: {window: oracle greedy tokens} already established for the SAME encoder output, weights and options
    (a previous gate_windows call's "oracle_tokens"); a window whose GPU tokens equal them is identical without
    another oracle pass."""
    from vlog_amd.metrics import edit_distance, normalize
    from vlog_amd.segments import split_segments_by_timestamps
    from oracle.decode import generate_one

    import time
    ws = list(range(len(results))) if windows is None else list(windows)
    ident, margins, ns_diff, non_ident = [], [], 0.0, []
    cum_diff = 0.0                      # worst |GPU cum_logprob - oracle teacher-forced sum| (relative to max(1, |sum|))
    oracle_tokens = {}
    t0 = time.time()
    todo = []
    for w in ws:
        if known is not None and w in known and list(results[w].tokens) == list(known[w]):
            ident.append(True)
            oracle_tokens[w] = list(known[w])
        else:
            todo.append(w)
    for c0 in range(0, len(todo), chunk):
        progress(f"gate_windows: {c0}/{len(todo)} windows checked, {time.time() - t0:.1f} s")
        cw = todo[c0:c0 + chunk]
        enc = enc_of(cw)
        toks = [list(results[w].tokens) for w in cw]
        ended = [len(prompt) + len(t) < opt.max_length for t in toks]
        for j, (w, (ms, ns, cum)) in enumerate(zip(cw, teacher_force_batch(orc, enc, prompt, toks, ended, st, opt))):
            same = bool(np.all(ms > 0.0))
            ident.append(same)
            ns_diff = max(ns_diff, abs(ns - float(results[w].no_speech_prob)))
            cg = getattr(results[w], "cum_logprob", None)
            if cg is not None and np.isfinite(cum):
                cum_diff = max(cum_diff, abs(float(cg) - cum) / max(1.0, abs(cum)))
            if same:
                oracle_tokens[w] = toks[j]
                margins.append(float(np.min(ms)) if ms.size else 0.0)
            else:
                non_ident.append(w)
                progress(f"gate_windows: window {w} not identical: oracle greedy re-decode")
                r = generate_one(orc, orc.cross_kv(enc[j:j + 1]), prompt, st, opt)
                oracle_tokens[w] = list(r.tokens)
    errs, n_ref, dt, seg_mismatch = 0, 0, 0.0, 0
    for w in ws:
        ref, hyp = normalize(tokenizer.decode(oracle_tokens[w])), normalize(tokenizer.decode(results[w].tokens))
        errs += edit_distance(ref, hyp)
        n_ref += len(ref)
        a = split_segments_by_timestamps(results[w].tokens, st.timestamp_begin, time_offset(w), 3000, 30.0, 0)[0]
        b = split_segments_by_timestamps(oracle_tokens[w], st.timestamp_begin, time_offset(w), 3000, 30.0, 0)[0]
        if len(a) != len(b):
            seg_mismatch += 1
            continue
        for x, y in zip(a, b):
            dt = max(dt, abs(x["start"] - y["start"]), abs(x["end"] - y["end"]))
    n = len(ws)
    return {"n": n, "identical": int(sum(ident)), "identical_frac": round(sum(ident) / max(n, 1), 5),
            "wer_delta": round(errs / max(n_ref, 1), 6), "segment_max_dt_s": round(dt, 4),
            "segment_count_mismatch": seg_mismatch, "max_no_speech_diff": ns_diff,
            "max_cum_logprob_rel_diff": cum_diff,
            "min_margin_identical_nats": round(min(margins), 3) if margins else None,
            "non_identical_windows": non_ident, "oracle_passes": len(todo),
            "oracle_tokens": oracle_tokens,
            "gates": {"identical_frac": GATE_IDENTICAL, "wer_delta": GATE_WER, "segment_dt_s": GATE_DT}}


GATE_CUM_REL = 2e-2        # the GPU's cumulative log-prob vs the oracle's teacher-forced sum (relative to max(1, |sum|))
GATE_NO_SPEECH = 1e-3      # no-speech probability


def assert_gates(g: dict) -> None:
    assert g["identical_frac"] >= GATE_IDENTICAL, g
    assert g["max_cum_logprob_rel_diff"] <= GATE_CUM_REL, g
    assert g["max_no_speech_diff"] <= GATE_NO_SPEECH, g
    assert g["wer_delta"] <= GATE_WER, g
    assert g["segment_max_dt_s"] <= GATE_DT + 1e-9, g
    assert g["segment_count_mismatch"] <= (1.0 - GATE_IDENTICAL) * g["n"], g
