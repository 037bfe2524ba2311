"""Word-alignment restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

CTranslate2 `Whisper.align` as faster-whisper `find_alignment` drives it [FW↑] (config 5,
word_timestamps=True), which follows openai `timing.find_alignment`:
  tokens  = sot_sequence + [<|notimestamps|>] + text_tokens + [<|endoftext|>]
  weights = cross-attention softmax of the alignment heads, cropped to num_frames // 2 keys and
            re-normalised, z-scored over the token axis, median-filtered (width 7) along time, head-averaged
  matrix  = weights[len(sot_sequence): -1]; (text_idx, time_idx) = DTW(-matrix)
  text_token_probs = softmax over the text vocabulary [0, eot) at each position, taken at the next token.
`median_filter` / `dtw` are pinned against transformers' `_median_filter` / `_dynamic_time_warping`
([TF] models/whisper/generation_whisper.py:43-116).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .decode import log_softmax


def median_filter(x: np.ndarray, width: int) -> np.ndarray:
    """Median over a sliding window along the last axis, reflect-padded (width odd)."""
    if width <= 0 or width % 2 != 1:
        raise ValueError("median filter width must be odd")
    pad = width // 2
    if x.shape[-1] <= pad:
        return x
    xp = np.pad(x, [(0, 0)] * (x.ndim - 1) + [(pad, pad)], mode="reflect")
    win = np.lib.stride_tricks.sliding_window_view(xp, width, axis=-1)
    return np.sort(win, axis=-1)[..., pad]


def dtw(x: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """openai dtw_cpu + backtrace on a cost matrix x [N, M] -> (text_indices, time_indices)."""
    N, M = x.shape
    cost = np.full((N + 1, M + 1), np.inf, dtype=np.float32)
    trace = -np.ones((N + 1, M + 1), dtype=np.float32)
    cost[0, 0] = 0
    for j in range(1, M + 1):
        for i in range(1, N + 1):
            c0, c1, c2 = cost[i - 1, j - 1], cost[i - 1, j], cost[i, j - 1]
            if c0 < c1 and c0 < c2:
                c, t = c0, 0
            elif c1 < c0 and c1 < c2:
                c, t = c1, 1
            else:
                c, t = c2, 2
            cost[i, j] = x[i - 1, j - 1] + c
            trace[i, j] = t
    i, j = N, M
    trace[0, :] = 2
    trace[:, 0] = 1
    path = []
    while i > 0 or j > 0:
        path.append((i - 1, j - 1))
        t = trace[i, j]
        if t == 0:
            i -= 1
            j -= 1
        elif t == 1:
            i -= 1
        elif t == 2:
            j -= 1
        else:
            raise RuntimeError("unexpected DTW trace")
    p = np.array(path[::-1])
    return p[:, 0], p[:, 1]


def alignment_matrix(attn: np.ndarray, num_frames: int, sot_len: int, medfilt_width: int = 7) -> np.ndarray:
    """attn [heads, n_tokens, 1500] softmax weights -> DTW input matrix [n_text + 1, num_frames // 2]."""
    w = attn[:, :, : num_frames // 2].astype(np.float64)
    w = w / w.sum(-1, keepdims=True)
    mean = w.mean(-2, keepdims=True)
    std = w.std(-2, keepdims=True)
    w = (w - mean) / std
    w = median_filter(w, medfilt_width)
    m = w.mean(0)
    return m[sot_len: -1]


def find_alignment(model, cross, sot_sequence: List[int], text_tokens: List[int], st, num_frames: int,
                   alignment_heads, medfilt_width: int = 7):
    """-> (text_token_probs [n_text], text_indices, time_indices) for one window (model = OracleWhisper)."""
    tokens = list(sot_sequence) + [st.no_timestamps] + list(text_tokens) + [st.eot]
    logits, _, cw = model.decode(np.asarray([tokens]), cross, return_cross_attn=True)
    sampled = logits[0, len(sot_sequence):, : st.eot]
    lp = log_softmax(sampled)
    probs = np.exp(lp[np.arange(len(text_tokens)), text_tokens])
    attn = np.stack([cw[l][0, h] for l, h in alignment_heads])          # [heads, n_tokens, 1500]
    m = alignment_matrix(attn, num_frames, len(sot_sequence), medfilt_width)
    ti, tj = dtw(-m)
    return probs, ti, tj
