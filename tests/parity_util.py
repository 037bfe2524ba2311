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
from dataclasses import asdict, dataclass
from typing import List, Sequence

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


def sample_indices(n: int, k: int) -> List[int]:
    """k window indices spread over [0, n), first and last included."""
    if k >= n:
        return list(range(n))
    return sorted({int(round(i * (n - 1) / (k - 1))) for i in range(k)})
