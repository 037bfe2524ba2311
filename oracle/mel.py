"""Log-mel restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Follows faster-whisper `FeatureExtractor.__call__` / `get_mel_filters` / `stft` [FW↑, 1.1.x], which the
reference reaches through `model.transcribe(str(wav), ...)` (`worker/transcription.py:105-111`):

  x        = pcm (float32, int16/32768 for the worker's s16le WAV)
  x        = pad(x, (0, 160))                         # faster-whisper >= 1.1 appends one hop of zeros
  frames   = reflect-centered STFT, n_fft 400, hop 160, periodic Hann (np.hanning(401)[:-1])
  power    = |X|^2, last STFT frame dropped            # -> N//160 + 1 frames
  mel      = slaney filterbank (0..8 kHz) @ power
  log_spec = log10(max(mel, 1e-10))
  log_spec = max(log_spec, log_spec.max() - 8)         # GLOBAL max over the whole file
  out      = (log_spec + 4) / 4

Computed in float64 (more accurate than the float32 upstream path); the GPU kernel is compared to it at
max-abs <= 1e-4 (BASELINE.json north_star).
"""
from __future__ import annotations

import numpy as np

N_FFT = 400
HOP = 160
SR = 16000


def mel_filters(n_mels: int, sr: int = SR, n_fft: int = N_FFT) -> np.ndarray:
    """faster-whisper `FeatureExtractor.get_mel_filters` (librosa slaney mel, slaney norm). [n_mels, 201]."""
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    min_mel, max_mel = 0.0, 45.245640471924965          # hz_to_mel(8000, slaney)
    mels = np.linspace(min_mel, max_mel, n_mels + 2)
    f_sp = 200.0 / 3
    freqs = f_sp * mels
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    log_t = mels >= min_log_mel
    freqs[log_t] = min_log_hz * np.exp(logstep * (mels[log_t] - min_log_mel))
    fdiff = np.diff(freqs)
    ramps = freqs.reshape(-1, 1) - fftfreqs.reshape(1, -1)
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    weights = np.maximum(0.0, np.minimum(lower, upper))
    enorm = 2.0 / (freqs[2: n_mels + 2] - freqs[:n_mels])
    return weights * enorm[:, None]


def hann_window(n_fft: int = N_FFT) -> np.ndarray:
    """Periodic Hann: np.hanning(n+1)[:-1]."""
    return np.hanning(n_fft + 1)[:-1]


def n_frames_for(n_samples: int, padding: int = HOP) -> int:
    """Number of mel frames faster-whisper produces for n_samples of audio (after the last-frame drop)."""
    return (n_samples + padding) // HOP


def power_spectrum(pcm: np.ndarray, padding: int = HOP) -> np.ndarray:
    """|STFT|^2 with the last frame dropped, float64 [201, n_frames]."""
    x = np.asarray(pcm, dtype=np.float32).astype(np.float64)
    if padding:
        x = np.pad(x, (0, padding))
    xp = np.pad(x, (N_FFT // 2, N_FFT // 2), mode="reflect")
    n_stft = 1 + (len(xp) - N_FFT) // HOP
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(n_stft)[:, None]
    frames = xp[idx] * hann_window()[None, :]
    spec = np.fft.rfft(frames, n=N_FFT, axis=-1)            # [n_stft, 201]
    power = (spec.real ** 2 + spec.imag ** 2).T               # [201, n_stft]
    return power[:, :-1]


def log_mel_unclamped(pcm: np.ndarray, n_mels: int, padding: int = HOP) -> np.ndarray:
    """log10(max(mel @ |X|^2, 1e-10)), float64 [n_mels, n_frames] — before the global clamp."""
    mel = mel_filters(n_mels) @ power_spectrum(pcm, padding)
    return np.log10(np.maximum(mel, 1e-10))


def clamp_and_scale(log_spec: np.ndarray, gmax: float | None = None) -> np.ndarray:
    if gmax is None:
        gmax = float(log_spec.max())
    return (np.maximum(log_spec, gmax - 8.0) + 4.0) / 4.0


def log_mel(pcm: np.ndarray, n_mels: int, padding: int = HOP) -> np.ndarray:
    """faster-whisper FeatureExtractor(audio): float32 [n_mels, (N+padding)//160]."""
    return clamp_and_scale(log_mel_unclamped(pcm, n_mels, padding)).astype(np.float32)


def pad_or_trim(mel: np.ndarray, length: int = 3000) -> np.ndarray:
    """faster-whisper `pad_or_trim` on the frame axis (zero pad on the right)."""
    if mel.shape[-1] > length:
        return mel[..., :length]
    if mel.shape[-1] < length:
        pad = [(0, 0)] * (mel.ndim - 1) + [(0, length - mel.shape[-1])]
        return np.pad(mel, pad)
    return mel
