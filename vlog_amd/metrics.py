"""Word error rate (own Levenshtein implementation; jiwer is not available) for the WER-delta metric."""
from __future__ import annotations

import re
from typing import List, Sequence


def normalize(text: str) -> List[str]:
    return re.sub(r"[^\w\s']", " ", text.lower()).split()


def edit_distance(a: Sequence, b: Sequence) -> int:
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def word_error_rate(reference: str, hypothesis: str) -> float:
    r, h = normalize(reference), normalize(hypothesis)
    if not r:
        return 0.0 if not h else 1.0
    return edit_distance(r, h) / len(r)
