"""Model weights: local HF-format directories and seeded synthetic weights.

The reference passes a model *name* (`WHISPER_MODEL`, `config.py:263`) that faster-whisper resolves by
downloading from the HF Hub (`worker/transcription.py:81-85`).  This engine never downloads anything:
`resolve_model()` maps

  * a local directory with `config.json` + `model.safetensors` (HF Whisper layout) -> those weights;
  * a local CTranslate2 directory (`model.bin`, the layout a faster-whisper deployment uses) -> its weights,
    dequantised to float32 (vlog_amd/ct2.py);
  * a name with `VLOG_AMD_MODEL_DIR_<name>` (or `VLOG_AMD_MODEL_ROOT/<name>`) set -> that directory;
  * `"synthetic:<name>[:seed]"` -> random-init weights of that architecture (there are no real
    checkpoints in this environment; BASELINE.md "Synthetic audio");

and raises a ValueError otherwise.

Synthetic init follows the upstream initialiser shape (normal(0, 0.02) for linear/conv/embedding weights,
sinusoids for the encoder positions) but gives biases and LayerNorm affines small random values so every
bias/affine path is exercised.  `eot_after` optionally plants one direction in the decoder positional
embedding and the <|endoftext|> embedding row so that greedy decoding ends after a speech-like number of
tokens instead of running to the 448-token limit (documented in DESIGN.md; both engines see identical
weights, so parity is unaffected).
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .dims import ModelDims, custom_dims, model_dims


def _gen(seed: int, name: str) -> torch.Generator:
    h = int.from_bytes(hashlib.sha256(f"{seed}:{name}".encode()).digest()[:8], "little") & ((1 << 63) - 1)
    g = torch.Generator(device="cpu")
    g.manual_seed(h)
    return g


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> torch.Tensor:
    inc = np.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-inc * torch.arange(channels // 2, dtype=torch.float64))
    t = torch.arange(length, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([torch.sin(t), torch.cos(t)], dim=1).float()


def weight_shapes(dims: ModelDims) -> Dict[str, Tuple[int, ...]]:
    d, f, m = dims.n_state, dims.n_ffn, dims.n_mels
    s: Dict[str, Tuple[int, ...]] = {
        "model.encoder.conv1.weight": (d, m, 3), "model.encoder.conv1.bias": (d,),
        "model.encoder.conv2.weight": (d, d, 3), "model.encoder.conv2.bias": (d,),
        "model.encoder.embed_positions.weight": (dims.n_audio_ctx, d),
        "model.encoder.layer_norm.weight": (d,), "model.encoder.layer_norm.bias": (d,),
        "model.decoder.embed_tokens.weight": (dims.n_vocab, d),
        "model.decoder.embed_positions.weight": (dims.n_text_ctx, d),
        "model.decoder.layer_norm.weight": (d,), "model.decoder.layer_norm.bias": (d,),
    }

    def attn(p):
        s.update({p + "q_proj.weight": (d, d), p + "q_proj.bias": (d,), p + "k_proj.weight": (d, d),
                  p + "v_proj.weight": (d, d), p + "v_proj.bias": (d,), p + "out_proj.weight": (d, d),
                  p + "out_proj.bias": (d,)})

    def ln(p):
        s.update({p + "weight": (d,), p + "bias": (d,)})

    def mlp(p):
        s.update({p + "fc1.weight": (f, d), p + "fc1.bias": (f,), p + "fc2.weight": (d, f), p + "fc2.bias": (d,)})

    for i in range(dims.n_enc_layer):
        p = f"model.encoder.layers.{i}."
        attn(p + "self_attn."); ln(p + "self_attn_layer_norm."); ln(p + "final_layer_norm."); mlp(p)
    for i in range(dims.n_dec_layer):
        p = f"model.decoder.layers.{i}."
        attn(p + "self_attn."); ln(p + "self_attn_layer_norm."); attn(p + "encoder_attn.")
        ln(p + "encoder_attn_layer_norm."); ln(p + "final_layer_norm."); mlp(p)
    return s


def synthetic_state_dict(dims: ModelDims, seed: int = 0, eot_after: Optional[int] = None,
                         std: float = 0.02) -> Dict[str, torch.Tensor]:
    """Seeded random-init weights (float32, CPU), HF naming.  Per-tensor generators make any subset
    reproducible on its own."""
    sd: Dict[str, torch.Tensor] = {}
    for name, shape in weight_shapes(dims).items():
        g = _gen(seed, name)
        if name == "model.encoder.embed_positions.weight":
            t = sinusoids(shape[0], shape[1])
        elif name.endswith("layer_norm.weight"):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name.endswith(".bias"):
            t = std * torch.randn(shape, generator=g)
        else:
            t = std * torch.randn(shape, generator=g)
        sd[name] = t.float()
    if eot_after is not None:
        plant_eot(sd, dims, eot_after, seed)
    return sd


# Final decoder residual-stream std of the seeded random init, by decoder depth (measured with the oracle on
# teacher-forced sequences; used to scale the planted <|endoftext|> ramp to the model's depth).
_RESID_STD = {4: 0.41, 6: 0.67, 12: 1.50, 24: 2.94, 32: 4.5}


def _resid_std(n_layers: int) -> float:
    ks = sorted(_RESID_STD)
    if n_layers in _RESID_STD:
        return _RESID_STD[n_layers]
    lo = max([k for k in ks if k <= n_layers], default=ks[0])
    hi = min([k for k in ks if k >= n_layers], default=ks[-1])
    if lo == hi:
        return _RESID_STD[lo] * n_layers / lo
    t = (n_layers - lo) / (hi - lo)
    return _RESID_STD[lo] * (1 - t) + _RESID_STD[hi] * t


EOT_KAPPA = 4.0


def plant_eot(sd: Dict[str, torch.Tensor], dims: ModelDims, eot_after: int, seed: int = 0) -> None:
    """Plant one direction u: E[<|endoftext|>] = c_e * u (the norm of a random row) and decoder position p
    carries slope * p * u with slope = EOT_KAPPA * s_L / (c_e * eot_after) (s_L = final residual std for this
    decoder depth), so the <|endoftext|> logit rises by about EOT_KAPPA over `eot_after` positions and
    greedy decoding ends near there."""
    d = dims.n_state
    g = _gen(seed, "plant_eot")
    u = torch.randn(d, generator=g)
    u = u / u.norm()
    pos = sd["model.decoder.embed_positions.weight"]
    c_e = 0.02 * float(np.sqrt(d))            # same norm as any random embedding row
    slope = EOT_KAPPA * _resid_std(dims.n_dec_layer) / (c_e * float(eot_after))
    pos += slope * torch.arange(pos.shape[0], dtype=torch.float32)[:, None] * u[None, :]
    sd["model.decoder.embed_tokens.weight"][dims.specials.eot] = c_e * u


def stored_as_bf16(name: str, t: torch.Tensor) -> bool:
    """Which tensors the engine keeps in bf16: weight matrices and conv kernels.  Biases, LayerNorm affines
    and the position tables stay float32 (vlog_amd/engine.py pack_weights)."""
    return name.endswith(".weight") and t.dim() >= 2 and "embed_positions" not in name


def round_bf16(sd: Dict[str, torch.Tensor]) -> Dict[str, np.ndarray]:
    """The values the GPU engine actually stores, as float32 numpy arrays for the oracle."""
    return {k: (v.to(torch.bfloat16).float() if stored_as_bf16(k, v) else v.float()).numpy() for k, v in sd.items()}


# ----------------------------------------------------------------------------- local model directories
def dims_from_hf_config(cfg: dict, name: str = "local") -> ModelDims:
    heads = ()
    if cfg.get("alignment_heads"):
        heads = tuple(tuple(x) for x in cfg["alignment_heads"])
    return custom_dims(name, cfg["num_mel_bins"], cfg["d_model"], cfg["encoder_attention_heads"],
                       cfg["encoder_layers"], cfg["decoder_layers"], cfg["vocab_size"],
                       cfg["vocab_size"] >= 51865, alignment_heads=heads)


def load_hf_dir(path: str) -> Tuple[ModelDims, Dict[str, torch.Tensor]]:
    from safetensors.torch import load_file

    with open(os.path.join(path, "config.json")) as f:
        cfg = json.load(f)
    dims = dims_from_hf_config(cfg, os.path.basename(os.path.normpath(path)))
    sd: Dict[str, torch.Tensor] = {}
    for fn in sorted(os.listdir(path)):
        if fn.endswith(".safetensors"):
            sd.update(load_file(os.path.join(path, fn)))
    sd = {k: v.float() for k, v in sd.items() if k.startswith("model.")}
    missing = set(weight_shapes(dims)) - set(sd)
    if missing:
        raise ValueError(f"{path}: missing weights {sorted(missing)[:5]} ...")
    return dims, sd


def load_model_dir(path: str) -> Tuple[ModelDims, Dict[str, torch.Tensor]]:
    """A local model directory: CTranslate2 (model.bin) or HF (config.json + *.safetensors)."""
    if os.path.isfile(os.path.join(path, "model.bin")):
        from .ct2 import load_ct2_dir
        dims, sd, _ = load_ct2_dir(path)
        return dims, sd
    return load_hf_dir(path)


def resolve_model(model_size_or_path: str, seed: int = 0, eot_after: Optional[int] = None
                  ) -> Tuple[ModelDims, Dict[str, torch.Tensor], Optional[str]]:
    """-> (dims, float32 CPU state dict, model directory or None)."""
    spec = model_size_or_path
    if spec.startswith("synthetic:"):
        parts = spec.split(":")
        name = parts[1]
        if len(parts) > 2:
            seed = int(parts[2])
        dims = model_dims(name)
        return dims, synthetic_state_dict(dims, seed, eot_after), None
    if os.path.isdir(spec):
        dims, sd = load_model_dir(spec)
        return dims, sd, spec
    env = os.environ.get("VLOG_AMD_MODEL_DIR_" + spec.replace("-", "_").replace(".", "_"))
    root = os.environ.get("VLOG_AMD_MODEL_ROOT")
    for cand in [env, os.path.join(root, spec) if root else None]:
        if cand and os.path.isdir(cand):
            dims, sd = load_model_dir(cand)
            return dims, sd, cand
    raise ValueError(
        f"model {spec!r}: no local weights (set VLOG_AMD_MODEL_DIR_<name> or VLOG_AMD_MODEL_ROOT, pass a "
        f"directory, or use 'synthetic:<name>'); downloading is not supported")
