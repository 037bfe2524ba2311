"""Host-side segment logic of the transcription path (faster-whisper `generate_segments` helpers [FW↑ 1.1.x]).

  split_segments_by_timestamps — `_split_segments_by_timestamps`: slice the token stream at consecutive
      timestamp pairs; start/end = window offset + (token - timestamp_begin) * 0.02 s; a single trailing
      timestamp means "no speech after it" (seek advances a whole window), otherwise seek moves to the last
      timestamp (2 mel frames per timestamp step).
  compression_ratio — len(utf8) / len(zlib(utf8)) (fallback trigger above 2.4).
  needs_fallback — the generate_with_fallback decision (compression ratio, avg logprob, silence exemption).
  avg_logprob — recovered from the CTranslate2 score: score * len**length_penalty / (len + 1).
"""
from __future__ import annotations

import zlib
from typing import List, Optional, Sequence, Tuple

TIME_PRECISION = 0.02
INPUT_STRIDE = 2


def split_segments_by_timestamps(tokens: Sequence[int], timestamp_begin: int, time_offset: float,
                                 segment_size: int, segment_duration: float, seek: int
                                 ) -> Tuple[List[dict], int, bool]:
    tokens = list(tokens)
    tb = timestamp_begin
    segs: List[dict] = []
    single_ending = len(tokens) >= 2 and tokens[-2] < tb <= tokens[-1]
    cuts = [i for i in range(1, len(tokens)) if tokens[i] >= tb and tokens[i - 1] >= tb]
    if cuts:
        if single_ending:
            cuts.append(len(tokens))
        last = 0
        for cut in cuts:
            piece = tokens[last:cut]
            segs.append(dict(seek=seek,
                             start=time_offset + (piece[0] - tb) * TIME_PRECISION,
                             end=time_offset + (piece[-1] - tb) * TIME_PRECISION,
                             tokens=piece))
            last = cut
        if single_ending:
            seek += segment_size
        else:
            seek += (tokens[last - 1] - tb) * INPUT_STRIDE
    else:
        duration = segment_duration
        stamps = [t for t in tokens if t >= tb]
        if stamps and stamps[-1] != tb:
            duration = (stamps[-1] - tb) * TIME_PRECISION
        segs.append(dict(seek=seek, start=time_offset, end=time_offset + duration, tokens=tokens))
        seek += segment_size
    return segs, seek, single_ending


def compression_ratio(text: str) -> float:
    b = text.encode("utf-8")
    return len(b) / len(zlib.compress(b)) if b else 0.0


def avg_logprob(score: float, n_tokens: int, length_penalty: float = 1.0) -> float:
    return score * (n_tokens ** length_penalty) / (n_tokens + 1)


def needs_fallback(comp_ratio: float, avg_lp: float, no_speech_prob: float,
                   compression_ratio_threshold: Optional[float] = 2.4, log_prob_threshold: Optional[float] = -1.0,
                   no_speech_threshold: Optional[float] = 0.6) -> Tuple[bool, bool]:
    """-> (needs_fallback, below_compression_threshold)."""
    fb = False
    below = True
    if compression_ratio_threshold is not None and comp_ratio > compression_ratio_threshold:
        fb = True
        below = False
    if log_prob_threshold is not None and avg_lp < log_prob_threshold:
        fb = True
    if (no_speech_threshold is not None and no_speech_prob > no_speech_threshold
            and log_prob_threshold is not None and avg_lp < log_prob_threshold):
        fb = False
    return fb, below


def should_skip_window(no_speech_prob: float, avg_lp: float, no_speech_threshold: Optional[float] = 0.6,
                       log_prob_threshold: Optional[float] = -1.0) -> bool:
    """faster-whisper's "no voice activity" skip after generate_with_fallback."""
    if no_speech_threshold is None:
        return False
    skip = no_speech_prob > no_speech_threshold
    if log_prob_threshold is not None and avg_lp > log_prob_threshold:
        skip = False
    return skip
