"""Word alignment glue (faster-whisper find_alignment -> CTranslate2 align [FW↑]); the arithmetic (cross-attention
capture, z-score, median filter, DTW) runs on the GPU in libwhisper_mi355 (csrc/align.hip)."""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def align_tokens(engine, dims, tokenizer, text_tokens: List[int], num_frames: int, median_filter_width: int = 7,
                 slot: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    heads = dims.default_alignment_heads()
    return engine.align(slot, tokenizer.sot_sequence, text_tokens, num_frames, heads, median_filter_width)
