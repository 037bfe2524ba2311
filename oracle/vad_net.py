"""Silero VAD v5 (16 kHz) network restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

The network faster-whisper runs for `vad_filter=True` [FW↑ 1.1.x vad.py `SileroVADModel.__call__`,
`get_speech_timestamps`] — reached from the reference worker's call (worker/transcription.py:110).  Silero is
a third-party model (snakers4/silero-vad v5, shipped by faster-whisper 1.1 as an encoder ONNX graph and a
decoder ONNX graph); neither the weights nor onnxruntime are in this image, so the restatement follows the
published v5 architecture:

  get_speech_timestamps:  audio padded with zeros by 512 - len % 512 (a whole window when len % 512 == 0)
  SileroVADModel:         window t = audio[512t : 512t+512]; its input is the previous window's last 64
                          samples (zeros for t = 0) followed by the window: 576 samples
  encoder (per window):   reflect-pad 64 on the right -> 640; STFT conv, basis [258][1][256], stride 128 ->
                          4 frames; magnitude sqrt(re^2 + im^2) of 129 bins;
                          conv(129->128, k3, p1) ReLU; conv(128->64, k3, s2, p1) ReLU;
                          conv(64->64, k3, s2, p1) ReLU; conv(64->128, k3, p1) ReLU  -> 128 features
  decoder (sequential):   LSTMCell(128, 128) with (h, c) = 0 at t = 0, gates (i, f, g, o);
                          p_t = sigmoid(conv1x1(ReLU(h_t)))

Computed in float64.  Parity unpinned against Silero itself (no weights or ONNX runtime here): the oracle
pins the GPU kernels (vad.hip) on seeded weights; the chunking state machine downstream is pinned separately
(tests/test_vad.py).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

WINDOW = 512
CONTEXT = 64


def pad_audio(audio: np.ndarray) -> np.ndarray:
    """faster-whisper get_speech_timestamps: np.pad(audio, (0, 512 - len % 512))."""
    return np.pad(np.asarray(audio, dtype=np.float32), (0, WINDOW - len(audio) % WINDOW))


def window_inputs(audio: np.ndarray) -> np.ndarray:
    """[n_win][576]: context (previous window's tail, zeros first) + window."""
    a = np.asarray(audio, dtype=np.float64)
    assert len(a) % WINDOW == 0
    w = a.reshape(-1, WINDOW)
    ctx = np.zeros((len(w), CONTEXT))
    ctx[1:] = w[:-1, -CONTEXT:]
    return np.concatenate([ctx, w], axis=1)


def _conv(x: np.ndarray, w: np.ndarray, b: np.ndarray, stride: int) -> np.ndarray:
    """x [B][cin][T], w [cout][cin][3], pad 1 -> [B][cout][T'] with ReLU."""
    B, cin, T = x.shape
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1)))
    To = (T + 2 - 3) // stride + 1
    cols = np.stack([xp[:, :, f * stride: f * stride + 3] for f in range(To)], axis=1)   # [B][To][cin][3]
    y = np.einsum("btik,oik->bot", cols, w.astype(np.float64)) + b.astype(np.float64)[None, :, None]
    return np.maximum(y, 0.0)


def encoder(x576: np.ndarray, wt: Dict[str, np.ndarray]) -> np.ndarray:
    """[n_win][576] -> [n_win][128] encoder features."""
    x = np.concatenate([x576, x576[:, 574:510:-1]], axis=1)            # reflect right by 64
    basis = wt["stft.forward_basis_buffer"][:, 0, :].astype(np.float64)   # [258][256]
    frames = np.stack([x[:, f * 128: f * 128 + 256] for f in range(4)], axis=1)   # [B][4][256]
    spec = np.einsum("bfk,rk->brf", frames, basis)                      # [B][258][4]
    mag = np.sqrt(spec[:, :129] ** 2 + spec[:, 129:] ** 2)
    h = mag
    for i, s in enumerate((1, 2, 2, 1)):
        h = _conv(h, wt[f"encoder.{i}.reparam_conv.weight"], wt[f"encoder.{i}.reparam_conv.bias"], s)
    return h[:, :, 0]


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def decoder(feats: np.ndarray, wt: Dict[str, np.ndarray]) -> np.ndarray:
    w_ih = wt["decoder.rnn.weight_ih"].astype(np.float64)
    w_hh = wt["decoder.rnn.weight_hh"].astype(np.float64)
    b = wt["decoder.rnn.bias_ih"].astype(np.float64) + wt["decoder.rnn.bias_hh"].astype(np.float64)
    hw = wt["decoder.decoder.2.weight"].reshape(-1).astype(np.float64)
    hb = float(wt["decoder.decoder.2.bias"].reshape(-1)[0])
    pre = feats @ w_ih.T + b
    h = np.zeros(128)
    c = np.zeros(128)
    out = np.empty(len(feats))
    for t in range(len(feats)):
        g = pre[t] + w_hh @ h
        i, f, gg, o = _sig(g[:128]), _sig(g[128:256]), np.tanh(g[256:384]), _sig(g[384:])
        c = f * c + i * gg
        h = o * np.tanh(c)
        out[t] = _sig(float(np.maximum(h, 0.0) @ hw) + hb)
    return out


def speech_probs(audio: np.ndarray, wt: Dict[str, np.ndarray]) -> np.ndarray:
    """SileroVADModel.__call__ on an audio length that is a multiple of 512."""
    return decoder(encoder(window_inputs(audio), wt), wt)
