"""ctypes binding of include/whisper_mi355.h (libwhisper_mi355.so, built in-tree by `make -C vlog_amd/csrc`).

There is no fallback: if the library is missing or fails to load, `load()` raises, so a GPU run can never
silently route through a CPU path.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VLOG_AMD_LIB") or os.path.join(_HERE, "libwhisper_mi355.so")
ABI_VERSION = 2

# Every entry point include/whisper_mi355.h declares (tests check the library exports all of them).
SYMBOLS = (
    "wm_create", "wm_destroy", "wm_last_error", "wm_abi_version", "wm_set_weight", "wm_weights_complete", "wm_weight_count", "wm_weight_info",
    "wm_logmel", "wm_logmel_finalize", "wm_encode", "wm_reserve", "wm_cross_kv", "wm_generate", "wm_forward",
    "wm_detect_language", "wm_frame_energy", "wm_pcm_from_s16", "wm_vad_probs", "wm_cross_fp8_quantize", "wm_align", "wm_align_batch", "wm_dtw", "wm_device_bytes", "wm_profile_classes", "wm_profile_name", "wm_profile", "wm_profile_select",
    "wm_profile_read", "wm_set_option", "wm_get_option", "wm_encoder_attention",
)


class ModelDimsC(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "n_mels", "n_state", "n_head", "n_enc_layer", "n_dec_layer", "n_vocab", "n_audio_ctx", "n_text_ctx",
        "eot", "sot", "no_speech", "no_timestamps", "timestamp_begin", "blank")]


class GenerateArgsC(C.Structure):
    _fields_ = [
        ("n_windows", C.c_int32), ("h_slots", C.POINTER(C.c_int32)), ("prompt_len", C.c_int32),
        ("h_prompts", C.POINTER(C.c_int32)), ("sot_index", C.c_int32), ("beam_size", C.c_int32),
        ("patience", C.c_float), ("length_penalty", C.c_float), ("max_length", C.c_int32),
        ("temperature", C.c_float), ("num_hypotheses", C.c_int32), ("seed", C.c_uint64),
        ("h_suppress", C.POINTER(C.c_int32)), ("n_suppress", C.c_int32), ("suppress_blank", C.c_int32),
        ("max_initial_timestamp_index", C.c_int32), ("with_timestamps", C.c_int32), ("check_every", C.c_int32),
        ("h_tokens", C.POINTER(C.c_int32)), ("h_lengths", C.POINTER(C.c_int32)), ("h_scores", C.POINTER(C.c_float)),
        ("h_cum_logprob", C.POINTER(C.c_float)), ("h_no_speech", C.POINTER(C.c_float)),
        ("h_steps", C.POINTER(C.c_int32)),
        # ABI 2
        ("max_rows", C.c_int32), ("compact", C.c_int32), ("h_token_logprobs", C.POINTER(C.c_float)),
        ("h_token_logprobs_other", C.POINTER(C.c_float)), ("h_stats", C.POINTER(C.c_int64)),
    ]


_lib: Optional[C.CDLL] = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load the HIP engine library (raises if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(path):
        raise RuntimeError(f"{path} not found: build it with `make -C vlog_amd/csrc` (or __graft_entry__.build())")
    lib = C.CDLL(path)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "wm_create": (C.c_int, [C.POINTER(ModelDimsC), i32, C.POINTER(vp)]),
        "wm_destroy": (None, [vp]),
        "wm_last_error": (C.c_char_p, []),
        "wm_abi_version": (i32, []),
        "wm_set_weight": (C.c_int, [vp, C.c_char_p, vp, i64, vp]),
        "wm_weights_complete": (i32, [vp]),
        "wm_weight_count": (i32, [vp]),
        "wm_weight_info": (C.c_int, [vp, i32, C.POINTER(C.c_char_p), C.POINTER(i64), C.POINTER(i32)]),
        "wm_logmel": (C.c_int, [vp, vp, i64, i64, i64, i32, vp, i64, vp, vp]),
        "wm_logmel_finalize": (C.c_int, [vp, vp, i64, i64, vp, C.POINTER(C.c_float), C.POINTER(C.c_float), vp]),
        "wm_encode": (C.c_int, [vp, vp, i64, C.POINTER(i32), C.POINTER(i32), i32, vp, vp]),
        "wm_reserve": (C.c_int, [vp, i32, i32, vp]),
        "wm_cross_kv": (C.c_int, [vp, vp, i32, i32, vp]),
        "wm_generate": (C.c_int, [vp, C.POINTER(GenerateArgsC), vp]),
        "wm_forward": (C.c_int, [vp, i32, C.POINTER(i32), i32, C.POINTER(i32), vp, i32, C.POINTER(i32), i32, vp, vp]),
        "wm_frame_energy": (C.c_int, [vp, vp, i64, i32, vp, vp]),
        "wm_detect_language": (C.c_int, [vp, i32, C.POINTER(i32), i32, i32, C.POINTER(C.c_float), vp]),
        "wm_vad_probs": (C.c_int, [vp, vp, vp, i64, vp, vp, vp]),
        "wm_pcm_from_s16": (C.c_int, [vp, vp, i64, vp, vp]),
        "wm_cross_fp8_quantize": (C.c_int, [vp, vp, i64, vp, vp, vp]),
        "wm_align": (C.c_int, [vp, i32, i32, C.POINTER(i32), i32, C.POINTER(i32), i32, C.POINTER(i32), i32, i32,
                               C.POINTER(C.c_float), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), vp]),
        "wm_align_batch": (C.c_int, [vp, i32, C.POINTER(i32), i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32),
                                     C.POINTER(i32), C.POINTER(i32), i32, i32, C.POINTER(C.c_float), C.POINTER(i64),
                                     C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), vp]),
        "wm_dtw": (C.c_int, [vp, vp, i32, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), vp]),
        "wm_device_bytes": (i64, [vp]),
        "wm_profile_classes": (i32, []),
        "wm_profile_name": (C.c_char_p, [i32]),
        "wm_profile": (C.c_int, [vp, i32]),
        "wm_profile_select": (C.c_int, [vp, C.c_uint32]),
        "wm_set_option": (C.c_int, [vp, C.c_char_p, i64]),
        "wm_get_option": (C.c_int, [vp, C.c_char_p, C.POINTER(i64)]),
        "wm_encoder_attention": (C.c_int, [vp, vp, vp, i32, i32, vp]),
        "wm_profile_read": (C.c_int, [vp, i32, C.POINTER(i64), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                      C.POINTER(C.c_double)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.wm_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libwhisper_mi355 ABI {lib.wm_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().wm_last_error()
        raise RuntimeError(f"{what} failed: {msg.decode(errors='replace') if msg else 'unknown error'}")
