"""WebVTT serialisation, byte-compatible with the worker's own writer.

The worker turns `segment.start/.end/.text` into captions with `generate_webvtt` / `format_timestamp`
(`worker/transcription.py:37-58`) and writes `VIDEOS_DIR/<slug>/captions.vtt` (`:377-381`).  The worker keeps
doing that itself when this engine is dropped in; this module gives the benchmark and tests the same bytes
(pinned by tests/golden/vtt_cases.json, generated from the reference function).  Quirks preserved:
seconds use "%06.3f" on `seconds % 60` (59.9996 -> "00:00:60.000"), hours are not truncated past two
digits, and text is stripped but inner newlines are kept.
"""
from __future__ import annotations

from typing import Iterable, Mapping


def format_timestamp(seconds: float) -> str:
    hours = int(seconds // 3600)
    minutes = int((seconds % 3600) // 60)
    return "%02d:%02d:%06.3f" % (hours, minutes, seconds % 60)


def generate_webvtt(segments: Iterable[Mapping]) -> str:
    parts = ["WEBVTT\n\n"]
    for n, seg in enumerate(segments, start=1):
        parts.append("%d\n%s --> %s\n%s\n\n" % (n, format_timestamp(seg["start"]), format_timestamp(seg["end"]),
                                              seg["text"].strip()))
    return "".join(parts)
