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


def window_parity(orc, enc_window: np.ndarray, prompt, res, st, opt: GenerateOptions, window: int) -> WindowParity:
    """res: vlog_amd.engine.GenResult of that window; enc_window [1500, d] float32 (the GPU's encoder output)."""
    cross = orc.cross_kv(enc_window[None])
    ended = len(prompt) + len(res.tokens) < opt.max_length
    chosen, best, score, ns = teacher_force(orc, cross, prompt, res.tokens, st, opt, ended)
    margin = chosen - best
    return WindowParity(window, len(res.tokens), bool(np.all(margin >= 0.0)), float(margin.min()) if margin.size else 0.0,
                        float(res.score), score, float(res.no_speech_prob), ns)


def record(name: str, rows: List[WindowParity], **extra) -> dict:
    """Summary dict; also appended as one JSON line to $VLOG_AMD_PARITY_OUT when that is set."""
    out = {"name": name, "n": len(rows), "identical": int(sum(r.identical for r in rows)),
           "min_margin": min((r.min_margin for r in rows), default=0.0),
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
