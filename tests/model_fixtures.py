"""Builder-written model-directory fixtures (test infrastructure): an HF Whisper directory (config.json +
model.safetensors), a CTranslate2 directory (model.bin written to the layout vlog_amd/ct2.py documents, plus
CTranslate2's config.json) and a byte-level BPE tokenizer.json built locally with `tokenizers`.  No real
checkpoint exists offline; the fixtures carry seeded synthetic weights, so a model loaded from a directory can
be compared with the same weights loaded as `synthetic:<name>:<seed>`."""
from __future__ import annotations

import json
import os
import struct
from typing import Dict

import numpy as np
import torch


def write_hf_dir(path: str, sd: Dict[str, torch.Tensor], dims) -> None:
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    cfg = {"model_type": "whisper", "num_mel_bins": dims.n_mels, "d_model": dims.n_state,
           "encoder_attention_heads": dims.n_head, "decoder_attention_heads": dims.n_head,
           "encoder_layers": dims.n_enc_layer, "decoder_layers": dims.n_dec_layer, "vocab_size": dims.n_vocab,
           "max_source_positions": dims.n_audio_ctx, "max_target_positions": dims.n_text_ctx}
    if dims.alignment_heads:
        cfg["alignment_heads"] = [list(h) for h in dims.alignment_heads]
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(path, "model.safetensors"))


def _wstr(f, s: str) -> None:
    b = s.encode("utf-8")
    f.write(struct.pack("<H", len(b) + 1))
    f.write(b + b"\0")


def ct2_variables(sd: Dict[str, torch.Tensor], dims) -> Dict[str, np.ndarray]:
    """HF-named weights -> CTranslate2 Whisper variable names (fused q|k|v and k|v projections)."""
    g = {k: v.float().numpy() for k, v in sd.items()}
    d = dims.n_state
    v: Dict[str, np.ndarray] = {"encoder/num_heads": np.array(dims.n_head, np.int16),
                                "decoder/num_heads": np.array(dims.n_head, np.int16)}
    for c in ("conv1", "conv2"):
        v[f"encoder/{c}/weight"] = g[f"model.encoder.{c}.weight"]
        v[f"encoder/{c}/bias"] = g[f"model.encoder.{c}.bias"]
    v["encoder/position_encodings/encodings"] = g["model.encoder.embed_positions.weight"]

    def ln(dst, src):
        v[dst + "/gamma"], v[dst + "/beta"] = g[src + ".weight"], g[src + ".bias"]

    def selfattn(dst, src):
        v[dst + "/linear_0/weight"] = np.concatenate([g[src + ".q_proj.weight"], g[src + ".k_proj.weight"],
                                                      g[src + ".v_proj.weight"]])
        v[dst + "/linear_0/bias"] = np.concatenate([g[src + ".q_proj.bias"], np.zeros(d, np.float32),
                                                    g[src + ".v_proj.bias"]])
        v[dst + "/linear_1/weight"], v[dst + "/linear_1/bias"] = g[src + ".out_proj.weight"], g[src + ".out_proj.bias"]

    def ffn(dst, src):
        v[dst + "/linear_0/weight"], v[dst + "/linear_0/bias"] = g[src + ".fc1.weight"], g[src + ".fc1.bias"]
        v[dst + "/linear_1/weight"], v[dst + "/linear_1/bias"] = g[src + ".fc2.weight"], g[src + ".fc2.bias"]

    for i in range(dims.n_enc_layer):
        s, t = f"model.encoder.layers.{i}", f"encoder/layer_{i}"
        selfattn(t + "/self_attention", s + ".self_attn")
        ln(t + "/self_attention/layer_norm", s + ".self_attn_layer_norm")
        ln(t + "/ffn/layer_norm", s + ".final_layer_norm")
        ffn(t + "/ffn", s)
    ln("encoder/layer_norm", "model.encoder.layer_norm")
    v["decoder/embeddings/weight"] = g["model.decoder.embed_tokens.weight"]
    v["decoder/position_encodings/encodings"] = g["model.decoder.embed_positions.weight"]
    for i in range(dims.n_dec_layer):
        s, t = f"model.decoder.layers.{i}", f"decoder/layer_{i}"
        selfattn(t + "/self_attention", s + ".self_attn")
        ln(t + "/self_attention/layer_norm", s + ".self_attn_layer_norm")
        a = s + ".encoder_attn"
        v[t + "/attention/linear_0/weight"], v[t + "/attention/linear_0/bias"] = g[a + ".q_proj.weight"], g[a + ".q_proj.bias"]
        v[t + "/attention/linear_1/weight"] = np.concatenate([g[a + ".k_proj.weight"], g[a + ".v_proj.weight"]])
        v[t + "/attention/linear_1/bias"] = np.concatenate([np.zeros(d, np.float32), g[a + ".v_proj.bias"]])
        v[t + "/attention/linear_2/weight"], v[t + "/attention/linear_2/bias"] = g[a + ".out_proj.weight"], g[a + ".out_proj.bias"]
        ln(t + "/attention/layer_norm", s + ".encoder_attn_layer_norm")
        ln(t + "/ffn/layer_norm", s + ".final_layer_norm")
        ffn(t + "/ffn", s)
    ln("decoder/layer_norm", "model.decoder.layer_norm")
    return v


def write_ct2_dir(path: str, sd: Dict[str, torch.Tensor], dims, weight_dtype: str = "float32") -> None:
    """weight_dtype: float32 | float16 | bfloat16 | int8 (2-D weights only, per-row scale = 127 / max|row|, as
    CTranslate2 quantises)."""
    os.makedirs(path, exist_ok=True)
    v = ct2_variables(sd, dims)
    ids = {np.dtype(np.float32): 0, np.dtype(np.int8): 1, np.dtype(np.int16): 2, np.dtype(np.int32): 3,
           np.dtype(np.float16): 4}
    out = []
    for name, a in v.items():
        if name.endswith("/weight") and a.ndim == 2 and weight_dtype != "float32":
            if weight_dtype == "int8":
                scale = 127.0 / np.maximum(np.abs(a).max(axis=1), 1e-12)
                out.append((name, np.clip(np.round(a * scale[:, None]), -127, 127).astype(np.int8), None))
                out.append((name + "_scale", scale.astype(np.float32), None))
                continue
            if weight_dtype == "float16":
                out.append((name, a.astype(np.float16), None))
                continue
            if weight_dtype == "bfloat16":
                u = a.astype(np.float32).view(np.uint32)
                out.append((name, ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16), 5))
                continue
        out.append((name, a, None))
    with open(os.path.join(path, "model.bin"), "wb") as f:
        f.write(struct.pack("<I", 6))
        _wstr(f, "WhisperSpec")
        f.write(struct.pack("<I", 3))
        f.write(struct.pack("<I", len(out)))
        for name, a, forced in out:
            _wstr(f, name)
            f.write(struct.pack("<B", a.ndim))
            for s in a.shape:
                f.write(struct.pack("<I", s))
            f.write(struct.pack("<B", forced if forced is not None else ids[a.dtype]))
            b = np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<")).tobytes()
            f.write(struct.pack("<I", len(b)))
            f.write(b)
        f.write(struct.pack("<I", 1))
        _wstr(f, "decoder/projection/weight")
        _wstr(f, "decoder/embeddings/weight")
    cfg = {"alignment_heads": [list(h) for h in dims.default_alignment_heads()],
           "suppress_ids": [], "suppress_ids_begin": [220, dims.specials.eot]}
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f)


def write_tokenizer_json(path: str, dims) -> None:
    """A byte-level BPE tokenizer.json with the Whisper special-token layout of `dims` (ids eot ..
    n_vocab - 1): 256 byte tokens, then unique pseudo-words, then the specials in id order."""
    from tokenizers import AddedToken, Tokenizer, decoders, models, pre_tokenizers
    from vlog_amd.tokenizer import _gpt2_byte_order, _special_texts

    order = _gpt2_byte_order()
    # GPT-2 bytes_to_unicode: printable bytes map to themselves, the rest to 256 + n
    printable = set(order[:188])
    b2u, n = {}, 0
    for b in range(256):
        if b in printable:
            b2u[b] = chr(b)
        else:
            b2u[b] = chr(256 + n)
            n += 1
    st = dims.specials
    vocab: Dict[str, int] = {}
    for i, b in enumerate(order):
        vocab[b2u[b]] = i
    rng = np.random.default_rng(4242)
    syl = ["ba", "ko", "ri", "tu", "me", "sa", "lo", "ni", "da", "ve", "shu", "tra"]
    i = len(vocab)
    while i < st.eot:
        w = ("Ġ" if rng.random() < 0.7 else "") + "".join(syl[int(k)] for k in rng.integers(0, len(syl), 3)) + str(i)
        if w not in vocab:
            vocab[w] = i
            i += 1
    tk = Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    specials = _special_texts(st, dims.n_vocab)
    tk.add_special_tokens([AddedToken(specials[k], special=True) for k in range(st.eot, dims.n_vocab)])
    assert tk.token_to_id("<|startoftranscript|>") == st.sot and tk.get_vocab_size() == dims.n_vocab
    tk.save(os.path.join(path, "tokenizer.json"))
