"""Opt-in `faster_whisper` overlay: put `<repo>/compat` on PYTHONPATH and the UNCHANGED vlog transcription worker
(`worker/transcription.py:78`: `from faster_whisper import WhisperModel`) runs on the MI355X engine.

Not on the default path, so a real faster-whisper install (the CPU baseline) can coexist in the same
environment.  The worker's literal `device="cpu", compute_type="int8"` (`worker/transcription.py:81-85`) is
remapped to the GPU (bf16) and logged; model names resolve to local directories only
(VLOG_AMD_MODEL_DIR_<name> / VLOG_AMD_MODEL_ROOT) or `synthetic:<name>` — nothing is downloaded.
"""
from __future__ import annotations

import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from vlog_amd.audio import load_audio as _load_audio  # noqa: E402
from vlog_amd.dims import known_models  # noqa: E402
from vlog_amd.transcribe import (  # noqa: E402,F401
    BatchedInferencePipeline,
    Segment,
    TranscriptionInfo,
    TranscriptionOptions,
    VadOptions,
    WhisperModel,
    Word,
)

__version__ = "1.1.1+vlog_amd"


def decode_audio(input_file, sampling_rate: int = 16000, split_stereo: bool = False):
    if split_stereo:
        raise NotImplementedError("split_stereo is not supported")
    return _load_audio(input_file, sampling_rate)


def available_models():
    return known_models()


def download_model(*args, **kwargs):
    raise RuntimeError("vlog_amd never downloads models: point VLOG_AMD_MODEL_DIR_<name> at a local directory")


def format_timestamp(seconds: float, always_include_hours: bool = False, decimal_marker: str = ".") -> str:
    """faster_whisper.utils.format_timestamp."""
    assert seconds >= 0, "non-negative timestamp expected"
    ms = round(seconds * 1000.0)
    hours, ms = divmod(ms, 3_600_000)
    minutes, ms = divmod(ms, 60_000)
    secs, ms = divmod(ms, 1_000)
    hours_marker = f"{hours:02d}:" if always_include_hours or hours > 0 else ""
    return f"{hours_marker}{minutes:02d}:{secs:02d}{decimal_marker}{ms:03d}"


__all__ = ["WhisperModel", "BatchedInferencePipeline", "decode_audio", "available_models", "download_model",
           "format_timestamp", "Segment", "Word", "TranscriptionInfo", "TranscriptionOptions", "VadOptions",
           "__version__"]
