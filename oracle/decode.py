"""Logit rules, greedy / beam / sampling search, language detection (TEST INFRASTRUCTURE ONLY).

Restates CTranslate2 `Whisper.generate` / `detect_language` as faster-whisper drives them from
`generate_with_fallback` / `detect_language` [FW↑ 1.1.x] (reference call `worker/transcription.py:105-111`):

  rules per step, in this order (openai `DecodingTask._get_logit_filters`, CT2 logits processors):
    1. SuppressBlank  — at the first sampled step suppress " " (blank) and <|endoftext|>
    2. SuppressTokens — the faster-whisper suppress list (config non-speech ids + special tokens)
    3. ApplyTimestampRules — pinned against transformers `WhisperTimeStampLogitsProcessor`
       ([TF] generation/logits_process.py:1909-2049): suppress <|notimestamps|>; pairs; monotonicity;
       first token a timestamp <= max_initial_timestamp_index; timestamp logsumexp > max text logprob
       forces a timestamp.
  greedy   — argmax of the rule-masked log-softmax; score = cumulative logprob (incl. <|endoftext|>)
             / len(tokens)**length_penalty (CT2 normalisation; faster-whisper recovers
             avg_logprob = score * len**lp / (len + 1)).
  beam     — openai `BeamSearchDecoder` semantics (each beam proposes its top beam+1 tokens; candidates are
             ranked by cumulative logprob; finished ones are collected until round(beam * patience);
             final choice by score / len**length_penalty).
  no_speech_prob — softmax of the raw logits at the <|startoftranscript|> position, token <|nospeech|>.
  max_length counts the prompt (faster-whisper passes max_length=448 and max_new_tokens + len(prompt)).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

NEG_INF = -np.inf


def log_softmax(x: np.ndarray) -> np.ndarray:
    """log-softmax over the last axis; a fully masked row (all -inf) stays all -inf (never NaN)."""
    x = np.asarray(x, dtype=np.float64)
    m = np.max(x, axis=-1, keepdims=True)
    live = np.isfinite(m)
    m = np.where(live, m, 0.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        out = x - m - np.log(np.sum(np.exp(x - m), axis=-1, keepdims=True))
    return np.where(live, out, -np.inf)


def apply_rules(logits: np.ndarray, sampled: Sequence[int], st, suppress_tokens: Sequence[int],
                suppress_blank: bool, max_initial_timestamp_index: Optional[int],
                with_timestamps: bool = True, force_timestamps: bool = True) -> np.ndarray:
    """logits [V] for ONE hypothesis; `sampled` = tokens generated after the prompt.  force_timestamps=False
    stops before the last rule (diagnostics: the logits the forcing decision is taken on)."""
    x = np.array(logits, dtype=np.float64, copy=True)
    first = len(sampled) == 0
    if suppress_blank and first:
        x[st.blank] = NEG_INF
        x[st.eot] = NEG_INF
    if len(suppress_tokens):
        x[np.asarray(suppress_tokens, dtype=np.int64)] = NEG_INF
    if not with_timestamps:
        return x
    tb = st.timestamp_begin
    x[st.no_timestamps] = NEG_INF
    last_ts = len(sampled) >= 1 and sampled[-1] >= tb
    pen_ts = len(sampled) < 2 or sampled[-2] >= tb
    if last_ts:
        if pen_ts:
            x[tb:] = NEG_INF
        else:
            x[: st.eot] = NEG_INF
    ts = [t for t in sampled if t >= tb]
    if ts:
        last = ts[-1] if (last_ts and not pen_ts) else ts[-1] + 1
        x[tb:last] = NEG_INF
    if first:
        x[:tb] = NEG_INF
        if max_initial_timestamp_index is not None:
            x[tb + max_initial_timestamp_index + 1:] = NEG_INF
    if not force_timestamps:
        return x
    lp = log_softmax(x)
    ts_lp = np.logaddexp.reduce(lp[tb:])
    if ts_lp > np.max(lp[:tb]):
        x[:tb] = NEG_INF
    return x


@dataclass
class GenerateResult:
    tokens: List[int]
    score: float
    no_speech_prob: float
    cum_logprob: float = 0.0
    all_hypotheses: List[List[int]] = field(default_factory=list)


@dataclass
class GenerateOptions:
    beam_size: int = 1
    patience: float = 1.0
    length_penalty: float = 1.0
    max_length: int = 448
    suppress_tokens: Sequence[int] = ()
    suppress_blank: bool = True
    max_initial_timestamp_index: Optional[int] = 50
    with_timestamps: bool = True
    sampling_temperature: float = 0.0
    num_hypotheses: int = 1
    seed: int = 0
    hyp_offset: int = 0        # sampling: index of this window's first hypothesis row in the engine's call


def _norm(cum: float, n: int, lp: float) -> float:
    return cum / (max(n, 1) ** lp)


def _prefill(model, cross, prompt: Sequence[int], st):
    toks = np.asarray([list(prompt)], dtype=np.int64)
    logits, cache = model.decode(toks, cross)
    no_speech = 0.0
    if st.sot in prompt:
        sot_idx = list(prompt).index(st.sot)
        p = np.exp(log_softmax(logits[0, sot_idx]))
        no_speech = float(p[st.no_speech])
    return logits[0, -1], cache, no_speech


def generate_one(model, cross, prompt: Sequence[int], st, opt: GenerateOptions) -> GenerateResult:
    """One window.  `cross` = model.cross_kv(enc[None]) for that window."""
    if opt.sampling_temperature > 0:
        return _sample(model, cross, prompt, st, opt)
    if opt.beam_size > 1:
        return _beam(model, cross, prompt, st, opt)
    last_logits, cache, no_speech = _prefill(model, cross, prompt, st)
    sampled: List[int] = []
    cum = 0.0
    pos = len(prompt)
    finished = False
    while pos < opt.max_length:
        x = apply_rules(last_logits, sampled, st, opt.suppress_tokens, opt.suppress_blank,
                        opt.max_initial_timestamp_index, opt.with_timestamps)
        lp = log_softmax(x)
        tok = int(np.argmax(lp))
        cum += float(lp[tok])
        if tok == st.eot:
            finished = True
            break
        sampled.append(tok)
        if pos + 1 >= opt.max_length:
            break
        logits, cache = model.decode(np.asarray([[tok]]), cross, cache, offset=pos)
        last_logits = logits[0, -1]
        pos += 1
    del finished
    return GenerateResult(sampled, _norm(cum, len(sampled), opt.length_penalty), no_speech, cum)


def _beam(model, cross, prompt, st, opt: GenerateOptions) -> GenerateResult:
    return beam_many(model, cross, prompt, st, opt)[0]


def beam_many(model, cross, prompt, st, opt: GenerateOptions, on_step=None) -> List[GenerateResult]:
    """Beam search over several windows in lockstep (`cross` = model.cross_kv(enc[W])): each window's beam
    bookkeeping is exactly the one-window search below; the decoder runs all W x K hypothesis rows at once
    (window-major, sharing their window's cross-attention K/V).  A finished window's rows keep decoding a dummy
    token that nothing reads."""
    K = opt.beam_size
    W = cross[0][0].shape[0]
    max_cand = int(round(K * opt.patience))
    toks = np.asarray([list(prompt)] * W, dtype=np.int64)
    logits, cache = model.decode(toks, cross)
    no_speech = [0.0] * W
    if st.sot in prompt:
        i = list(prompt).index(st.sot)
        no_speech = [float(np.exp(log_softmax(logits[w, i]))[st.no_speech]) for w in range(W)]
    # replicate each window's prefill state for its K beams (window-major rows)
    cache = [(np.repeat(k, K, 0), np.repeat(v, K, 0)) for k, v in cache]
    logits_rows = np.repeat(logits[:, -1], K, 0)
    seqs = [[[] for _ in range(K)] for _ in range(W)]
    sums = [np.array([0.0] + [NEG_INF] * (K - 1)) for _ in range(W)]   # only beam 0 is live at the first step
    finished = [dict() for _ in range(W)]
    done = [False] * W
    pos = len(prompt)
    while not all(done):
        src_all = np.arange(W * K)
        last = np.full(W * K, st.eot, dtype=np.int64)
        pos += 1
        if on_step is not None:
            on_step(pos, sum(done))
        for w in range(W):
            if done[w]:
                continue
            cands = []
            for j in range(K):
                if not np.isfinite(sums[w][j]):
                    continue
                x = apply_rules(logits_rows[w * K + j], seqs[w][j], st, opt.suppress_tokens, opt.suppress_blank,
                                opt.max_initial_timestamp_index, opt.with_timestamps)
                lp = log_softmax(x)
                top = np.argsort(-lp, kind="stable")[: K + 1]
                for t in top:
                    cands.append((sums[w][j] + lp[t], j, int(t)))
            cands.sort(key=lambda c: -c[0])
            new_seqs, new_src, new_sums, new_fin = [], [], [], []
            for score, j, t in cands:
                if t == st.eot:
                    new_fin.append((score, tuple(seqs[w][j])))
                else:
                    new_seqs.append(seqs[w][j] + [t]); new_src.append(j); new_sums.append(score)
                    if len(new_seqs) == K:
                        break
            for score, sq in new_fin:
                if len(finished[w]) >= max_cand:
                    break
                finished[w].setdefault(sq, score)
            if len(finished[w]) >= max_cand or pos >= opt.max_length or not new_seqs:
                if len(finished[w]) < K:
                    for score, sq in sorted(zip(new_sums, new_seqs), key=lambda z: -z[0]):
                        if len(finished[w]) >= K:
                            break
                        finished[w].setdefault(tuple(sq), score)
                done[w] = True
                continue
            while len(new_seqs) < K:
                new_seqs.append(list(new_seqs[0])); new_src.append(new_src[0]); new_sums.append(NEG_INF)
            src_all[w * K:(w + 1) * K] = w * K + np.asarray(new_src)
            last[w * K:(w + 1) * K] = [sq[-1] for sq in new_seqs]
            seqs[w] = new_seqs
            sums[w] = np.asarray(new_sums)
        if all(done):
            break
        cache = [(k[src_all], v[src_all]) for k, v in cache]
        logits, cache = model.decode(last[:, None], cross, cache, offset=pos - 1)
        logits_rows = logits[:, -1]
    out = []
    for w in range(W):
        ranked = sorted(finished[w].items(), key=lambda kv: -_norm(kv[1], len(kv[0]), opt.length_penalty))
        best, cum = ranked[0]
        out.append(GenerateResult(list(best), _norm(cum, len(best), opt.length_penalty), no_speech[w], cum,
                                  [list(sq) for sq, _ in ranked]))
    return out


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def gumbel_noise(seed: int, hyp: int, step: int, V: int) -> np.ndarray:
    """Counter-based Gumbel noise of the engine's sampling (vlog_amd/csrc/search.hip `gumbel`): for token i,
    u = ((h >> 41) + 0.5) / 2^23 with h = mix64(seed ^ mix64(hyp << 40 ^ step << 20 ^ i)), g = -log(-log(u)) in
    float32 (u is exact and strictly inside (0, 1)).  Keyed on (call seed, hypothesis row, decode step, token), so a draw does not depend on batch
    composition or launch order.  (faster-whisper samples with CTranslate2's own RNG [FW↑]: the draws are
    this build's, the sampling rule — argmax of logits / T + Gumbel noise = a draw from softmax(logits / T) —
    is the same.)"""
    i = np.arange(V, dtype=np.uint64)
    key = (np.uint64(hyp) << np.uint64(40)) ^ (np.uint64(step) << np.uint64(20)) ^ i
    h = _mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ _mix64(key))
    u = ((h >> np.uint64(41)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 8388608.0)
    return -np.log(-np.log(u))


def _sample(model, cross, prompt, st, opt: GenerateOptions) -> GenerateResult:
    """Sampling at temperature T (faster-whisper best_of = num_hypotheses): Gumbel-max over the rule-masked
    logits / T with the engine's counter-based noise; the best hypothesis by cum_logprob / len**lp."""
    results = []
    for j in range(max(1, opt.num_hypotheses)):
        last_logits, cache, no_speech = _prefill(model, cross, prompt, st)
        sampled, cum, pos = [], 0.0, len(prompt)
        step = 0
        while pos < opt.max_length:
            x = apply_rules(last_logits, sampled, st, opt.suppress_tokens, opt.suppress_blank,
                            opt.max_initial_timestamp_index, opt.with_timestamps)
            lp = log_softmax(x)
            keys = x / opt.sampling_temperature + gumbel_noise(opt.seed, opt.hyp_offset + j, step, x.shape[0])
            tok = int(np.argmax(keys))
            step += 1
            cum += float(lp[tok])
            if tok == st.eot:
                break
            sampled.append(tok)
            if pos + 1 >= opt.max_length:
                break
            logits, cache = model.decode(np.asarray([[tok]]), cross, cache, offset=pos)
            last_logits = logits[0, -1]
            pos += 1
        results.append(GenerateResult(sampled, _norm(cum, len(sampled), opt.length_penalty), no_speech, cum))
    results.sort(key=lambda r: -r.score)
    return results[0]


def detect_language(model, cross, st) -> List[tuple]:
    """CT2 `detect_language`: one step from [sot]; softmax restricted to the language tokens.
    -> [(code, prob)] sorted by probability (descending)."""
    logits, _ = model.decode(np.asarray([[st.sot]]), cross)
    lang = logits[0, 0, st.lang_begin: st.lang_begin + st.n_langs].astype(np.float64)
    p = np.exp(log_softmax(lang))
    order = np.argsort(-p, kind="stable")
    return [(st.lang_codes[i], float(p[i])) for i in order]


def score_sequence(model, cross, prompt: Sequence[int], tokens: Sequence[int], st, opt: GenerateOptions,
                   ended_with_eot: bool = True):
    """Teacher-force `tokens` (generated, no eot) through the oracle with the same rules.
    -> (chosen_logprobs, best_logprobs, normalised_score): per step the rule-masked log-prob of the chosen
    token (eot appended if `ended_with_eot`) and the best log-prob at that step, plus cum/len**lp."""
    seq = list(tokens) + ([st.eot] if ended_with_eot else [])
    toks = np.asarray([list(prompt) + list(tokens)])
    logits, _ = model.decode(toks, cross)
    P = len(prompt)
    chosen, best = [], []
    for i, t in enumerate(seq):
        x = apply_rules(logits[0, P - 1 + i], list(tokens[:i]), st, opt.suppress_tokens, opt.suppress_blank,
                        opt.max_initial_timestamp_index, opt.with_timestamps)
        lp = log_softmax(x)
        chosen.append(float(lp[t]))
        best.append(float(np.max(lp)))
    cum = float(np.sum(chosen))
    return np.array(chosen), np.array(best), _norm(cum, len(tokens), opt.length_penalty)
