"""Audio input: RIFF/WAVE s16le reader (the worker's ffmpeg output format) and a seeded speech-like generator.

The worker extracts `pcm_s16le`, 16 kHz, mono WAV with ffmpeg (`worker/transcription.py:276-292`) and passes
the path to `transcribe` (`:105`); faster-whisper decodes it to float32 = int16 / 32768 [FW↑].  `load_audio`
does the same for WAV files (no ffmpeg/PyAV in this environment; other containers raise ValueError).

`speech_like(seconds, seed)` is the BASELINE.md synthetic source: glottal pulse train 90-250 Hz with
jitter, 3 moving formants per 150-300 ms syllable, unvoiced noise bursts, pauses 0.2-3 s, RMS about
-26 dBFS, int16-quantised.  `numpy.random.default_rng(seed)`; corpora concatenate clips with seed = index.
"""
from __future__ import annotations

import io
import struct
import wave
from typing import Union

import numpy as np
from scipy.signal import lfilter

SR = 16000


def load_audio(src: Union[str, bytes, io.IOBase], sampling_rate: int = SR) -> np.ndarray:
    """WAV (PCM s16le/s32le/u8, mono or multi-channel, 16 kHz) -> float32 mono in [-1, 1)."""
    if isinstance(src, (bytes, bytearray)):
        src = io.BytesIO(src)
    try:
        with wave.open(src, "rb") as w:
            ch, width, rate, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
            raw = w.readframes(n)
    except (wave.Error, EOFError) as e:
        raise ValueError(f"unsupported audio container (only RIFF/WAVE PCM is decoded here): {e}") from None
    if width == 2:
        x = np.frombuffer(raw, dtype="<i2").astype(np.float32) / 32768.0
    elif width == 4:
        x = np.frombuffer(raw, dtype="<i4").astype(np.float32) / 2147483648.0
    elif width == 1:
        x = (np.frombuffer(raw, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"unsupported sample width {width}")
    if ch > 1:
        x = x.reshape(-1, ch).mean(axis=1)
    if rate != sampling_rate:
        raise ValueError(f"sample rate {rate} Hz; the engine expects {sampling_rate} Hz (the worker's ffmpeg -ar 16000)")
    return np.ascontiguousarray(x, dtype=np.float32)


def write_wav(path_or_buf, pcm: np.ndarray, sr: int = SR) -> None:
    x = np.asarray(pcm)
    if x.dtype != np.int16:
        x = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    with wave.open(path_or_buf, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(x.astype("<i2").tobytes())


def _resonator(f: float, bw: float, sr: int = SR):
    r = np.exp(-np.pi * bw / sr)
    th = 2 * np.pi * f / sr
    return [1.0 - r], [1.0, -2 * r * np.cos(th), r * r]


def speech_like(seconds: float, seed: int = 0, sr: int = SR, as_int16: bool = False) -> np.ndarray:
    rng = np.random.default_rng(seed)
    n_total = int(round(seconds * sr))
    out = np.zeros(n_total, dtype=np.float64)
    pos = int(rng.integers(0, int(0.3 * sr)))
    while pos < n_total:
        r = rng.random()
        if r < 0.12:                                 # pause (>= 2 s ones exercise VAD-style gaps)
            pos += int(rng.uniform(0.2, 3.0 if rng.random() < 0.3 else 0.8) * sr)
            continue
        dur = rng.uniform(0.15, 0.30)
        n = int(dur * sr)
        if pos + n > n_total:
            n = n_total - pos
        if n <= 16:
            break
        t = np.arange(n) / sr
        if rng.random() < 0.2:                       # unvoiced burst (fricative-like)
            nb = min(n, int(rng.uniform(0.05, 0.12) * sr))
            noise = rng.standard_normal(nb)
            b, a = _resonator(rng.uniform(3000, 6000), 1500)
            seg = lfilter(b, a, noise) * 0.3
            out[pos: pos + nb] += seg
            pos += nb + int(rng.uniform(0.01, 0.05) * sr)
            continue
        f0 = rng.uniform(90, 250)
        vib = 1 + 0.03 * np.sin(2 * np.pi * rng.uniform(3, 6) * t) + 0.01 * rng.standard_normal(n).cumsum() / np.sqrt(n)
        phase = np.cumsum(f0 * vib / sr)
        src = np.diff(np.floor(phase), prepend=0.0)          # one impulse per glottal period
        src = lfilter([1.0], [1.0, -0.95], src)               # glottal roll-off
        seg = np.zeros(n)
        for (lo, hi, bw) in ((300, 900, 80), (900, 2500, 120), (2400, 3500, 200)):
            fa, fb = rng.uniform(lo, hi), rng.uniform(lo, hi)
            k = 4
            edges = np.linspace(0, n, k + 1).astype(int)
            for j in range(k):                                  # piecewise-static moving formant
                fj = fa + (fb - fa) * (j + 0.5) / k
                b, a = _resonator(fj, bw)
                seg[edges[j]: edges[j + 1]] += lfilter(b, a, src[edges[j]: edges[j + 1]])
        env = np.sin(np.pi * np.linspace(0, 1, n)) ** 0.5
        out[pos: pos + n] += seg * env * rng.uniform(0.5, 1.0)
        pos += n + int(rng.uniform(0.0, 0.06) * sr)
    rms = np.sqrt(np.mean(out ** 2)) + 1e-12
    out *= (10 ** (-26 / 20)) / rms
    x16 = np.clip(np.round(out * 32768.0), -32768, 32767).astype(np.int16)
    return x16 if as_int16 else x16.astype(np.float32) / 32768.0


def room_tone(seconds: float, seed: int = 0, sr: int = SR, dbfs: float = -70.0, as_int16: bool = False) -> np.ndarray:
    """Silence as a recording has it: low-level pink-ish room noise at `dbfs` RMS (int16-quantised like
    speech_like), e.g. the gaps between the parts of a long-form programme."""
    rng = np.random.default_rng(10_000_019 + seed)
    n = int(round(seconds * sr))
    x = lfilter([1.0], [1.0, -0.9], rng.standard_normal(n))
    x *= (10 ** (dbfs / 20)) / (np.sqrt(np.mean(x ** 2)) + 1e-12)
    x16 = np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16)
    return x16 if as_int16 else x16.astype(np.float32) / 32768.0


QUIET_EVERY = 10


def long_form_window(i: int, seconds: float = 30.0) -> np.ndarray:
    """Window i of the variable-length corpus (bench.py --workload variable, the variable gates): speech_like(seed i),
    except every QUIET_EVERY-th window (i % QUIET_EVERY == QUIET_EVERY - 1) is room tone, so the corpus holds the
    near-empty windows (silence between programme parts) real long-form audio has."""
    if i % QUIET_EVERY == QUIET_EVERY - 1:
        return room_tone(seconds, i)
    return speech_like(seconds, i)


def corpus(n_clips: int, clip_seconds: float = 30.0, seed0: int = 0) -> np.ndarray:
    """Concatenation of n_clips speech-like clips with seeds seed0 .. seed0+n_clips-1 (float32)."""
    return np.concatenate([speech_like(clip_seconds, seed0 + i) for i in range(n_clips)])
