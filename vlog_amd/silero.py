"""Silero VAD v5 (16 kHz) network on the MI355X — the speech-probability model behind faster-whisper's
`vad_filter=True` [FW↑ vad.py `SileroVADModel`, `get_speech_timestamps`], reached from the reference worker's
call (worker/transcription.py:110).

The weights ship inside faster-whisper's package (an ONNX file) and are not in this image, so the network runs
with either
  * a local weights file (`.safetensors` or `.npz`) holding the Silero v5 JIT state-dict tensors under the
    names in `WEIGHT_SHAPES` (a maintainer exports them once from the public checkpoint), or
  * `synthetic:<seed>` — seeded random weights with the real STFT basis (Hann-windowed DFT), for tests and
    benches.
The product computes on the device only (libwhisper_mi355 `wm_vad_probs`; vad.hip); oracle/vad_net.py is the
CPU restatement the tests compare it with.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional

import numpy as np
import torch

WINDOW = 512
CONTEXT = 64

PREFIX = "_model."
WEIGHT_SHAPES = {
    "stft.forward_basis_buffer": (258, 1, 256),
    "encoder.0.reparam_conv.weight": (128, 129, 3), "encoder.0.reparam_conv.bias": (128,),
    "encoder.1.reparam_conv.weight": (64, 128, 3), "encoder.1.reparam_conv.bias": (64,),
    "encoder.2.reparam_conv.weight": (64, 64, 3), "encoder.2.reparam_conv.bias": (64,),
    "encoder.3.reparam_conv.weight": (128, 64, 3), "encoder.3.reparam_conv.bias": (128,),
    "decoder.rnn.weight_ih": (512, 128), "decoder.rnn.weight_hh": (512, 128),
    "decoder.rnn.bias_ih": (512,), "decoder.rnn.bias_hh": (512,),
    "decoder.decoder.2.weight": (1, 128, 1), "decoder.decoder.2.bias": (1,),
}


def stft_basis(n_fft: int = 256) -> np.ndarray:
    """[2*(n_fft/2+1), 1, n_fft]: rows k of the real DFT (cos) then the imaginary part (-sin), times a periodic
    Hann window — the fixed conv basis Silero's STFT module holds."""
    n = np.arange(n_fft)
    k = np.arange(n_fft // 2 + 1)[:, None]
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / n_fft)
    ang = 2 * np.pi * k * n / n_fft
    return np.concatenate([np.cos(ang) * win, -np.sin(ang) * win]).astype(np.float32)[:, None, :]


def synthetic_weights(seed: int = 0) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    w: Dict[str, np.ndarray] = {}
    for name, shape in WEIGHT_SHAPES.items():
        if name == "stft.forward_basis_buffer":
            w[name] = stft_basis()
            continue
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 128
        # gains chosen so speech-level audio spreads the output over (0, 1) instead of pinning it at 0.5
        gain = {"encoder.0.reparam_conv.weight": 0.5, "decoder.rnn.weight_ih": 4.0,
                "decoder.decoder.2.weight": -8.0}.get(name, 1.41 if name.startswith("encoder") and
                                                     name.endswith("weight") else 1.0)
        w[name] = (rng.standard_normal(shape) * (gain / np.sqrt(fan_in))).astype(np.float32)
    return w


def load_weights(path: str) -> Dict[str, np.ndarray]:
    """A local `.safetensors` / `.npz` file; names with or without the JIT `_model.` prefix."""
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        raw = load_file(path)
    elif path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            raw = {k: z[k] for k in z.files}
    else:
        raise ValueError(f"Silero VAD weights must be .safetensors or .npz: {path}")
    out: Dict[str, np.ndarray] = {}
    for k, v in raw.items():
        k = k[len(PREFIX):] if k.startswith(PREFIX) else k
        if k in WEIGHT_SHAPES:
            out[k] = np.asarray(v, dtype=np.float32)
    missing = [k for k in WEIGHT_SHAPES if k not in out]
    if missing:
        raise ValueError(f"Silero VAD weights {path}: missing {missing}")
    for k, shape in WEIGHT_SHAPES.items():
        if out[k].shape != shape:
            raise ValueError(f"Silero VAD weights {path}: {k} has shape {out[k].shape}, expected {shape}")
    return out


def resolve_weights(spec: str) -> Dict[str, np.ndarray]:
    if spec.startswith("synthetic"):
        parts = spec.split(":")
        return synthetic_weights(int(parts[1]) if len(parts) > 1 and parts[1] else 0)
    if not os.path.isfile(spec):
        raise FileNotFoundError(f"Silero VAD weights not found: {spec}")
    return load_weights(spec)


class _VadWeights(C.Structure):
    _fields_ = [("stft_basis", C.c_void_p), ("conv_w", C.c_void_p * 4), ("conv_b", C.c_void_p * 4),
                ("w_ih", C.c_void_p), ("w_hh", C.c_void_p), ("b_ih", C.c_void_p), ("b_hh", C.c_void_p),
                ("head_w", C.c_void_p), ("head_b", C.c_void_p)]


class SileroVad:
    """Device-resident Silero v5 weights + `__call__(audio) -> per-512-sample speech probabilities`, the
    contract of faster-whisper 1.1 `SileroVADModel.__call__` (audio length a multiple of 512)."""

    def __init__(self, engine, weights: Dict[str, np.ndarray]):
        self.engine = engine
        dev = engine.device
        self.t = {k: torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)).to(dev) for k, v in weights.items()}
        p = lambda k: self.t[k].data_ptr()  # noqa: E731
        s = _VadWeights()
        s.stft_basis = p("stft.forward_basis_buffer")
        for i in range(4):
            s.conv_w[i] = p(f"encoder.{i}.reparam_conv.weight")
            s.conv_b[i] = p(f"encoder.{i}.reparam_conv.bias")
        s.w_ih, s.w_hh = p("decoder.rnn.weight_ih"), p("decoder.rnn.weight_hh")
        s.b_ih, s.b_hh = p("decoder.rnn.bias_ih"), p("decoder.rnn.bias_hh")
        s.head_w, s.head_b = p("decoder.decoder.2.weight"), p("decoder.decoder.2.bias")
        self._w = s

    @classmethod
    def from_spec(cls, engine, spec: str) -> "SileroVad":
        return cls(engine, resolve_weights(spec))

    def probs_device(self, pcm: torch.Tensor) -> torch.Tensor:
        """pcm: f32 device tensor, length a multiple of 512 -> f32 device tensor of window probabilities."""
        from . import _capi
        n = int(pcm.numel())
        if n % WINDOW:
            raise ValueError("Silero VAD input length must be a multiple of 512")
        nw = n // WINDOW
        out = torch.empty(nw, dtype=torch.float32, device=pcm.device)
        if nw == 0:
            return out
        work = torch.empty(nw * 512, dtype=torch.float32, device=pcm.device)
        eng = self.engine
        _capi.check(eng.lib.wm_vad_probs(eng.h, C.byref(self._w), C.c_void_p(pcm.data_ptr()), n,
                                         C.c_void_p(work.data_ptr()), C.c_void_p(out.data_ptr()), eng.stream_ptr()),
                    "wm_vad_probs")
        return out

    def __call__(self, audio: np.ndarray) -> np.ndarray:
        dev = self.engine.device
        pcm = torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)).to(dev)
        out = self.probs_device(pcm)
        torch.cuda.synchronize(dev)
        return out.cpu().numpy()


def default_spec() -> Optional[str]:
    v = os.environ.get("VLOG_AMD_SILERO_VAD", "")
    return v or None
