"""CTranslate2 `model.bin` reader for Whisper models (the format faster-whisper loads [FW↑]).

The worker passes `WHISPER_MODEL` ("medium" by default, reference `config.py:263`) to
`WhisperModel(...)` (`worker/transcription.py:81-85`); in a faster-whisper deployment that name resolves to a
CTranslate2 model directory: `model.bin`, CTranslate2's `config.json` (alignment heads, suppress ids, language
ids) and `tokenizer.json` / `vocabulary.*`.  This module reads such a directory into the engine's HF-named
float32 state dict (vlog_amd/weights.py), so a local faster-whisper model directory drops in unchanged.

`model.bin` layout (CTranslate2 `ModelSpec._serialize`, binary version 5/6, restated from the published
source; CTranslate2 is not installed here, so this reader is pinned only by tests/model_fixtures.py, a writer of
the same layout — "parity unpinned" against real CTranslate2 output):

    u32 binary_version                 (>= 5 carries the alias table)
    str spec_name                      str := u16 length-including-NUL, bytes, NUL
    u32 spec_revision
    u32 n_variables, then n x { str name; u8 rank; u32 dims[rank]; u8 dtype; u32 nbytes; bytes data }
    u32 n_aliases,   then n x { str alias; str variable_name }

dtype ids: 0 float32, 1 int8, 2 int16, 3 int32, 4 float16, 5 bfloat16.  int8 weights carry a per-row
`<name>_scale` (float32) with w = q / scale.  Whisper variable names (ctranslate2/specs/whisper_spec.py):
encoder/{conv1,conv2}/{weight,bias}, encoder/position_encodings/encodings, encoder/layer_norm/{gamma,beta},
encoder/layer_<i>/self_attention/{layer_norm/*, linear_0 (fused q|k|v), linear_1 (out)},
encoder/layer_<i>/ffn/{layer_norm/*, linear_0 (fc1), linear_1 (fc2)}; decoder/embeddings/weight,
decoder/position_encodings/encodings, decoder/layer_norm/*, decoder/layer_<i>/self_attention/* (as the
encoder's), decoder/layer_<i>/attention/{layer_norm/*, linear_0 (q), linear_1 (fused k|v), linear_2 (out)},
decoder/layer_<i>/ffn/*; decoder/projection/weight aliases the embeddings.
"""
from __future__ import annotations

import json
import os
import re
import struct
from typing import BinaryIO, Dict, Tuple

import numpy as np
import torch

from .dims import ModelDims, custom_dims

DTYPES = {0: np.float32, 1: np.int8, 2: np.int16, 3: np.int32, 4: np.float16, 5: "bfloat16"}


def _read_str(f: BinaryIO) -> str:
    (n,) = struct.unpack("<H", f.read(2))
    b = f.read(n)
    if len(b) != n or not b.endswith(b"\0"):
        raise ValueError("model.bin: malformed string")
    return b[:-1].decode("utf-8")


def read_model_bin(path: str) -> Tuple[str, int, Dict[str, np.ndarray]]:
    """-> (spec name, spec revision, {variable name: array}); aliases resolved to their target arrays,
    bfloat16 variables returned as float32."""
    variables: Dict[str, np.ndarray] = {}
    with open(path, "rb") as f:
        (version,) = struct.unpack("<I", f.read(4))
        if version < 3 or version > 6:
            raise ValueError(f"{path}: unsupported CTranslate2 binary version {version}")
        spec = _read_str(f)
        (revision,) = struct.unpack("<I", f.read(4))
        (n_var,) = struct.unpack("<I", f.read(4))
        for _ in range(n_var):
            name = _read_str(f)
            (rank,) = struct.unpack("<B", f.read(1))
            shape = struct.unpack(f"<{rank}I", f.read(4 * rank)) if rank else ()
            (dt,) = struct.unpack("<B", f.read(1))
            (nbytes,) = struct.unpack("<I", f.read(4))
            data = f.read(nbytes)
            if len(data) != nbytes:
                raise ValueError(f"{path}: truncated variable {name}")
            if dt not in DTYPES:
                raise ValueError(f"{path}: variable {name} has unknown dtype id {dt}")
            if DTYPES[dt] == "bfloat16":
                u = np.frombuffer(data, dtype="<u2").astype(np.uint32) << 16
                arr = u.view(np.float32)
            else:
                arr = np.frombuffer(data, dtype=np.dtype(DTYPES[dt]).newbyteorder("<"))
            variables[name] = arr.reshape(shape) if shape else arr.reshape(())
        if version >= 5:
            (n_alias,) = struct.unpack("<I", f.read(4))
            for _ in range(n_alias):
                alias, target = _read_str(f), _read_str(f)
                variables[alias] = variables[target]
    return spec, revision, variables


def _dequant(v: Dict[str, np.ndarray], name: str) -> np.ndarray:
    w = v[name]
    if w.dtype == np.int8:
        scale = v.get(name + "_scale")
        if scale is None:
            raise ValueError(f"int8 variable {name} without {name}_scale")
        s = np.asarray(scale, dtype=np.float32)
        return w.astype(np.float32) / (s.reshape(-1, *([1] * (w.ndim - 1))) if s.ndim else s)
    return np.asarray(w, dtype=np.float32)


def dims_from_variables(v: Dict[str, np.ndarray], cfg: dict, name: str) -> ModelDims:
    d, n_mels = v["encoder/conv1/weight"].shape[:2]

    def n_layers(side):
        pat = re.compile(rf"^{side}/layer_(\d+)/")
        return len({m.group(1) for m in map(pat.match, v) if m})

    n_enc, n_dec = n_layers("encoder"), n_layers("decoder")
    n_head = int(v["encoder/num_heads"]) if "encoder/num_heads" in v else d // 64
    vocab = v["decoder/embeddings/weight"].shape[0]
    heads = cfg.get("alignment_heads") or ()
    return custom_dims(name, int(n_mels), int(d), n_head, n_enc, n_dec, int(vocab), vocab >= 51865,
                       alignment_heads=heads)


def to_hf_state_dict(v: Dict[str, np.ndarray], dims: ModelDims) -> Dict[str, torch.Tensor]:
    """CTranslate2 Whisper variables -> the engine's HF-named float32 state dict (fused projections split,
    k biases zero, int8 dequantised)."""
    d = dims.n_state
    sd: Dict[str, np.ndarray] = {}

    def lin(dst, src, bias=True):
        sd[dst + ".weight"] = _dequant(v, src + "/weight")
        if bias:
            sd[dst + ".bias"] = np.asarray(v[src + "/bias"], dtype=np.float32)

    def ln(dst, src):
        sd[dst + ".weight"] = np.asarray(v[src + "/gamma"], dtype=np.float32)
        sd[dst + ".bias"] = np.asarray(v[src + "/beta"], dtype=np.float32)

    def fused(dst_names, src, parts):
        w = _dequant(v, src + "/weight")
        b = np.asarray(v[src + "/bias"], dtype=np.float32) if (src + "/bias") in v else np.zeros(w.shape[0], np.float32)
        for i, n in enumerate(dst_names):
            sd[n + ".weight"] = w[i * d: (i + 1) * d]
            if parts[i]:
                sd[n + ".bias"] = b[i * d: (i + 1) * d]

    for c in ("conv1", "conv2"):
        lin(f"model.encoder.{c}", f"encoder/{c}")
    sd["model.encoder.embed_positions.weight"] = np.asarray(v["encoder/position_encodings/encodings"], np.float32)
    for i in range(dims.n_enc_layer):
        s, t = f"encoder/layer_{i}", f"model.encoder.layers.{i}"
        fused([f"{t}.self_attn.q_proj", f"{t}.self_attn.k_proj", f"{t}.self_attn.v_proj"],
              f"{s}/self_attention/linear_0", (True, False, True))
        lin(f"{t}.self_attn.out_proj", f"{s}/self_attention/linear_1")
        ln(f"{t}.self_attn_layer_norm", f"{s}/self_attention/layer_norm")
        ln(f"{t}.final_layer_norm", f"{s}/ffn/layer_norm")
        lin(f"{t}.fc1", f"{s}/ffn/linear_0")
        lin(f"{t}.fc2", f"{s}/ffn/linear_1")
    ln("model.encoder.layer_norm", "encoder/layer_norm")
    sd["model.decoder.embed_tokens.weight"] = _dequant(v, "decoder/embeddings/weight")
    sd["model.decoder.embed_positions.weight"] = np.asarray(v["decoder/position_encodings/encodings"], np.float32)
    for i in range(dims.n_dec_layer):
        s, t = f"decoder/layer_{i}", f"model.decoder.layers.{i}"
        fused([f"{t}.self_attn.q_proj", f"{t}.self_attn.k_proj", f"{t}.self_attn.v_proj"],
              f"{s}/self_attention/linear_0", (True, False, True))
        lin(f"{t}.self_attn.out_proj", f"{s}/self_attention/linear_1")
        ln(f"{t}.self_attn_layer_norm", f"{s}/self_attention/layer_norm")
        lin(f"{t}.encoder_attn.q_proj", f"{s}/attention/linear_0")
        w = _dequant(v, f"{s}/attention/linear_1/weight")
        b = np.asarray(v[f"{s}/attention/linear_1/bias"], np.float32)
        sd[f"{t}.encoder_attn.k_proj.weight"], sd[f"{t}.encoder_attn.v_proj.weight"] = w[:d], w[d:]
        sd[f"{t}.encoder_attn.v_proj.bias"] = b[d:]
        lin(f"{t}.encoder_attn.out_proj", f"{s}/attention/linear_2")
        ln(f"{t}.encoder_attn_layer_norm", f"{s}/attention/layer_norm")
        ln(f"{t}.final_layer_norm", f"{s}/ffn/layer_norm")
        lin(f"{t}.fc1", f"{s}/ffn/linear_0")
        lin(f"{t}.fc2", f"{s}/ffn/linear_1")
    ln("model.decoder.layer_norm", "decoder/layer_norm")
    return {k: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)) for k, a in sd.items()}


def load_ct2_dir(path: str) -> Tuple[ModelDims, Dict[str, torch.Tensor], dict]:
    """A CTranslate2 Whisper model directory -> (dims, HF-named float32 state dict, CT2 config.json dict)."""
    cfg = {}
    cp = os.path.join(path, "config.json")
    if os.path.isfile(cp):
        with open(cp) as f:
            cfg = json.load(f)
    spec, _, v = read_model_bin(os.path.join(path, "model.bin"))
    if "whisper" not in spec.lower():
        raise ValueError(f"{path}: model.bin holds a {spec!r} model, not Whisper")
    dims = dims_from_variables(v, cfg, os.path.basename(os.path.normpath(path)))
    return dims, to_hf_state_dict(v, dims), cfg
