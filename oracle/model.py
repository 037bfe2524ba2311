"""Whisper encoder/decoder forward in numpy (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates what CTranslate2's `models.Whisper.encode` / `generate` compute [FW↑] (the reference reaches them
through `worker/transcription.py:105-111`).  The architecture is pinned against transformers 5.15.0
`WhisperForConditionalGeneration` ([TF] `models/whisper/modeling_whisper.py:241-798`) on identical seeded
weights (tests/test_oracle_model.py):

  encoder: conv1(k3,p1)+GELU(erf), conv2(k3,s2,p1)+GELU, + sinusoidal positions, L x pre-LN block
           (MHA non-causal, k_proj without bias; MLP d->4d->d GELU), final LN (eps 1e-5)
  decoder: token embedding + learned positions, L x pre-LN block (causal self-attn with KV cache,
           cross-attn over the 1500 encoder positions, MLP), final LN, logits = h @ E^T (tied)

Weights are a dict in HF naming (vlog_amd/weights.py produces it); the computation runs in float32 (or
float64) on whatever values are given — the GPU engine stores the same values in bf16, so tests feed the
oracle the bf16-rounded weights.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np
from scipy.special import erf


def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round float32 values to bfloat16 (round-to-nearest-even) and return them as float32 (the definition, in
    integer arithmetic on the bit pattern)."""
    x32 = np.ascontiguousarray(x, dtype=np.float32)
    u = x32.view(np.uint32)
    # finite values: u <= 0xFF7FFFFF, so u + 0x8000 cannot wrap in uint32
    r = ((u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) & np.uint32(0xFFFF0000)).view(np.float32)
    return np.where(np.isfinite(x32), r, x32)


def to_bf16(x: np.ndarray) -> np.ndarray:
    """to_bf16_bits, computed by PyTorch's CPU float32 -> bfloat16 conversion (the same round-to-nearest-even,
    multithreaded: the oracle's bf16-activation mode rounds every activation, and the numpy form was half the
    oracle's time at large-v3 sizes).  tests/test_oracle_model.py pins the two forms bit for bit."""
    try:
        import torch
    except ImportError:                     # pragma: no cover - torch is part of this image
        return to_bf16_bits(x)
    x32 = np.ascontiguousarray(x, dtype=np.float32)
    return torch.from_numpy(x32).to(torch.bfloat16).float().numpy()


_POOL = None


def _threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:                  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def par_rows(fn, *arrays, min_rows: int = 2):
    """fn applied to slices of the leading axis of `arrays` on a thread pool, results concatenated on axis 0.
    Only for computations that are independent per leading index (numpy's elementwise ufuncs and batched
    matmul release the GIL and run single-threaded; the result is identical to fn(*arrays))."""
    global _POOL
    n = arrays[0].shape[0]
    k = min(_threads(), n // max(1, min_rows))
    if k <= 1:
        return fn(*arrays)
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(max_workers=_threads())
    cuts = [n * i // k for i in range(k + 1)]
    parts = list(_POOL.map(lambda i: fn(*(a[cuts[i]:cuts[i + 1]] for a in arrays)), range(k)))
    if isinstance(parts[0], tuple):
        return tuple(None if parts[0][j] is None else np.concatenate([p[j] for p in parts], axis=0)
                     for j in range(len(parts[0])))
    return np.concatenate(parts, axis=0)


def _gelu(x: np.ndarray) -> np.ndarray:
    return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)).astype(x.dtype))


def gelu(x: np.ndarray) -> np.ndarray:
    return par_rows(_gelu, x) if x.ndim >= 2 and x.size >= (1 << 20) else _gelu(x)


def layer_norm(x: np.ndarray, w: np.ndarray, b: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * w + b


def softmax(x: np.ndarray, axis: int = -1) -> np.ndarray:
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Encoder positional table (openai `sinusoids`; [TF] WhisperEncoder embed_positions init)."""
    inc = np.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2))
    t = np.arange(length)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1)


def conv1d(x: np.ndarray, w: np.ndarray, b: np.ndarray, stride: int) -> np.ndarray:
    """x [B, Cin, T], w [Cout, Cin, 3], padding 1 -> [B, Cout, T_out]."""
    B, Cin, T = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1)))
    T_out = (T + 2 - 3) // stride + 1
    cols = np.stack([xp[:, :, k: k + stride * (T_out - 1) + 1: stride] for k in range(3)], axis=-1)  # [B,Cin,Tout,3]
    cols = cols.transpose(0, 2, 1, 3).reshape(B, T_out, Cin * 3)
    y = cols @ w.reshape(w.shape[0], Cin * 3).T + b                                              # [B,Tout,Cout]
    return y.transpose(0, 2, 1)


class OracleWhisper:
    """`bf16_acts=True` restates the engine's numeric format in the DECODER: activations are rounded to
    bf16 exactly where libwhisper_mi355 stores them (LayerNorm outputs, q/k/v and the KV caches, attention
    outputs, GELU outputs, cross K/V), with float32 accumulation everywhere else — so a token-identity test
    compares the same arithmetic up to summation order instead of bf16 vs f32 rounding."""

    def __init__(self, sd: Dict[str, np.ndarray], dims, dtype=np.float32, bf16_acts: bool = False,
                 bf16_enc: bool = False):
        self.dims = dims
        self.bf16 = bf16_acts
        self.bf16_enc = bf16_enc
        self.dtype = dtype
        self.w = {k: np.asarray(v, dtype=dtype) for k, v in sd.items()}
        self.H = dims.n_head
        self.hd = dims.n_state // dims.n_head

    # ---------------------------------------------------------------- helpers
    def _q(self, x):
        return to_bf16(x) if self.bf16 else x

    def _lin(self, x, name, bias=True):
        y = x @ self.w[name + ".weight"].T
        if bias and (name + ".bias") in self.w:
            y = y + self.w[name + ".bias"]
        return y

    def _split(self, x):  # [B, T, d] -> [B, H, T, hd]
        B, T, _ = x.shape
        return x.reshape(B, T, self.H, self.hd).transpose(0, 2, 1, 3)

    def _merge(self, x):  # [B, H, T, hd] -> [B, T, d]
        B, H, T, hd = x.shape
        return x.transpose(0, 2, 1, 3).reshape(B, T, H * hd)

    def _attn(self, q, k, v, mask=None, return_weights=False):
        s = (q @ np.swapaxes(k, -1, -2)) / np.sqrt(self.hd).astype(self.dtype)
        if mask is not None:
            s = s + mask
        # the softmax is elementwise per row: sliced over a thread pool (numpy's ufuncs are single-threaded);
        # the matmuls stay on the calling thread (BLAS threads itself)
        p = par_rows(softmax, s) if s.size >= (1 << 20) else softmax(s, -1)
        o = p @ v
        return (o, p) if return_weights else (o, None)

    # ---------------------------------------------------------------- encoder
    def encode(self, mel: np.ndarray) -> np.ndarray:
        """mel [B, n_mels, 3000] -> [B, 1500, d]."""
        if self.bf16_enc:
            return self._encode_bf16(mel)
        w = self.w
        x = np.asarray(mel, dtype=self.dtype)
        x = gelu(conv1d(x, w["model.encoder.conv1.weight"], w["model.encoder.conv1.bias"], 1))
        x = gelu(conv1d(x, w["model.encoder.conv2.weight"], w["model.encoder.conv2.bias"], 2))
        x = x.transpose(0, 2, 1) + w["model.encoder.embed_positions.weight"][: x.shape[2]]
        for i in range(self.dims.n_enc_layer):
            p = f"model.encoder.layers.{i}."
            h = layer_norm(x, w[p + "self_attn_layer_norm.weight"], w[p + "self_attn_layer_norm.bias"])
            q = self._split(self._lin(h, p + "self_attn.q_proj"))
            k = self._split(self._lin(h, p + "self_attn.k_proj", bias=False))
            v = self._split(self._lin(h, p + "self_attn.v_proj"))
            o, _ = self._attn(q, k, v)
            x = x + self._lin(self._merge(o), p + "self_attn.out_proj")
            h = layer_norm(x, w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"])
            x = x + self._lin(gelu(self._lin(h, p + "fc1")), p + "fc2")
        return layer_norm(x, w["model.encoder.layer_norm.weight"], w["model.encoder.layer_norm.bias"])

    def _attn_enc_bf16(self, q, k, v):
        """Encoder self-attention in the engine's numeric format (libwhisper_mi355 attn_enc_v2_kernel): Q
        pre-scaled by 1/sqrt(64)*log2(e) and rounded to bf16, S = Q K^T in f32, P = exp2(S - rowmax) rounded to
        bf16 for the P.V product, the normaliser summed from the unrounded P, output rounded to bf16."""
        qs = to_bf16(q * np.float32(0.125 * 1.4426950408889634))
        s = qs @ k.transpose(0, 1, 3, 2)
        p = np.exp2(s - s.max(-1, keepdims=True))
        l = p.sum(-1, keepdims=True)
        return to_bf16((to_bf16(p) @ v) / l)

    def _encode_bf16(self, mel: np.ndarray) -> np.ndarray:
        """The encoder with the engine's rounding points (vlog_amd/csrc/engine.cpp encode_chunk): the im2col'd
        mel, the conv1 output, every LayerNorm output, q/k/v, the attention output and the GELU(fc1) output are
        stored as bf16; the residual stream and every accumulation stay float32."""
        w = self.w
        q_ = to_bf16
        x = q_(np.asarray(mel, dtype=np.float32))
        x = q_(gelu(conv1d(x, w["model.encoder.conv1.weight"], w["model.encoder.conv1.bias"], 1)))
        x = gelu(conv1d(x, w["model.encoder.conv2.weight"], w["model.encoder.conv2.bias"], 2))
        x = (x.transpose(0, 2, 1) + w["model.encoder.embed_positions.weight"][: x.shape[2]]).astype(np.float32)
        for i in range(self.dims.n_enc_layer):
            p = f"model.encoder.layers.{i}."
            h = q_(layer_norm(x, w[p + "self_attn_layer_norm.weight"], w[p + "self_attn_layer_norm.bias"]))
            q = self._split(q_(self._lin(h, p + "self_attn.q_proj")))
            k = self._split(q_(self._lin(h, p + "self_attn.k_proj", bias=False)))
            v = self._split(q_(self._lin(h, p + "self_attn.v_proj")))
            o = self._attn_enc_bf16(q, k, v)
            x = x + self._lin(self._merge(o), p + "self_attn.out_proj")
            h = q_(layer_norm(x, w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"]))
            x = x + self._lin(q_(gelu(self._lin(h, p + "fc1"))), p + "fc2")
        return q_(layer_norm(x, w["model.encoder.layer_norm.weight"], w["model.encoder.layer_norm.bias"]))

    # ---------------------------------------------------------------- decoder
    def cross_kv(self, enc: np.ndarray) -> List[Tuple[np.ndarray, np.ndarray]]:
        out = []
        enc = self._q(np.asarray(enc, dtype=self.dtype))
        for i in range(self.dims.n_dec_layer):
            p = f"model.decoder.layers.{i}.encoder_attn."
            k = self._q(self._lin(enc, p + "k_proj", bias=False))
            v = self._q(self._lin(enc, p + "v_proj"))
            out.append((self._split(k), self._split(v)))
        return out

    def decode(self, tokens: np.ndarray, cross: List[Tuple[np.ndarray, np.ndarray]],
               cache: Optional[List[Tuple[np.ndarray, np.ndarray]]] = None, offset: int = 0,
               return_cross_attn: bool = False):
        """tokens [B, L] (positions offset..offset+L-1) -> (logits [B, L, V] float, new cache[, cross weights])."""
        w = self.w
        B, L = tokens.shape
        x = w["model.decoder.embed_tokens.weight"][tokens] + w["model.decoder.embed_positions.weight"][offset: offset + L]
        Ltot = offset + L
        mask = np.triu(np.full((L, Ltot), -np.inf, dtype=self.dtype), k=offset + 1)
        new_cache = []
        cross_w = []
        for i in range(self.dims.n_dec_layer):
            p = f"model.decoder.layers.{i}."
            h = self._q(layer_norm(x, w[p + "self_attn_layer_norm.weight"], w[p + "self_attn_layer_norm.bias"]))
            q = self._split(self._q(self._lin(h, p + "self_attn.q_proj")))
            k = self._split(self._q(self._lin(h, p + "self_attn.k_proj", bias=False)))
            v = self._split(self._q(self._lin(h, p + "self_attn.v_proj")))
            if cache is not None and offset > 0:
                k = np.concatenate([cache[i][0], k], axis=2)
                v = np.concatenate([cache[i][1], v], axis=2)
            new_cache.append((k, v))
            o, _ = self._attn(q, k, v, mask)
            x = x + self._lin(self._q(self._merge(o)), p + "self_attn.out_proj")
            h = self._q(layer_norm(x, w[p + "encoder_attn_layer_norm.weight"], w[p + "encoder_attn_layer_norm.bias"]))
            q = self._split(self._q(self._lin(h, p + "encoder_attn.q_proj")))
            ck, cv = cross[i]
            if ck.shape[0] not in (1, B):   # hypotheses sharing their window's cross-KV (beam search): rows are
                # window-major groups of `rep`; broadcast each window's K/V over its group without a copy
                nw = ck.shape[0]
                rep = B // nw
                qg = q.reshape(nw, rep, *q.shape[1:])
                o, pw = self._attn(qg, ck[:, None], cv[:, None], return_weights=return_cross_attn)
                o = o.reshape(B, *o.shape[2:])
                pw = pw.reshape(B, *pw.shape[2:]) if pw is not None else None
            else:
                o, pw = self._attn(q, ck, cv, return_weights=return_cross_attn)
            if return_cross_attn:
                cross_w.append(pw)
            x = x + self._lin(self._q(self._merge(o)), p + "encoder_attn.out_proj")
            h = self._q(layer_norm(x, w[p + "final_layer_norm.weight"], w[p + "final_layer_norm.bias"]))
            x = x + self._lin(self._q(gelu(self._lin(h, p + "fc1"))), p + "fc2")
        x = self._q(layer_norm(x, w["model.decoder.layer_norm.weight"], w["model.decoder.layer_norm.bias"]))
        logits = x @ w["model.decoder.embed_tokens.weight"].T
        if return_cross_attn:
            return logits, new_cache, cross_w
        return logits, new_cache
