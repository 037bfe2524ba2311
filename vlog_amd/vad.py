"""Voice-activity filtering for `transcribe(..., vad_filter=True)` — the reference worker's call
(`worker/transcription.py:110`).

faster-whisper runs Silero VAD (ONNX) and then a fixed chunking state machine [FW↑ vad.py
`get_speech_timestamps`, `collect_chunks`, `restore_speech_timestamps` / `SpeechTimestampsMap`].  The
state machine, padding and timestamp restoration are restated exactly here.  The per-512-sample speech
probability comes from
  * the Silero v5 network on the GPU (vlog_amd/silero.py, libwhisper_mi355 `wm_vad_probs`) when the model was
    given Silero weights (WhisperModel(vad_model=...) / VLOG_AMD_SILERO_VAD) — on the audio padded exactly as
    faster-whisper pads it; or
  * without weights (they are not in this image), a GPU frame-energy kernel (`wm_frame_energy`) mapped through
    a logistic above the file's noise floor — a documented stand-in whose chunk boundaries do not match
    Silero's ("parity unpinned").
"""
from __future__ import annotations

import bisect
from typing import Iterable, List

import numpy as np
import torch

WINDOW = 512


def speech_probs(audio, model) -> np.ndarray:
    """audio: float32 numpy array, or a device tensor (streaming ingest keeps the PCM on the GPU)."""
    net = getattr(model, "vad_net", None)
    if net is not None:
        pad = WINDOW - len(audio) % WINDOW                         # faster-whisper pads a whole window at % == 0
        if isinstance(audio, torch.Tensor):
            a = torch.cat([audio.to(net.engine.device, torch.float32), audio.new_zeros(pad, dtype=torch.float32)])
            out = net.probs_device(a.contiguous())
            return out.cpu().numpy()
        a = np.asarray(audio, dtype=np.float32)
        return net(np.pad(a, (0, pad)))
    if isinstance(audio, torch.Tensor):
        db = model.engine.frame_energy_db(audio.to(torch.float32), WINDOW)
        finite = db[db > -100.0]
        floor = float(np.percentile(finite, 10)) if finite.size else -100.0
        thr = max(floor + 12.0, -55.0)
        return 1.0 / (1.0 + np.exp(-(db - thr) / 2.0))
    db = model.engine.frame_energy_db(torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)), WINDOW)
    finite = db[db > -100.0]
    floor = float(np.percentile(finite, 10)) if finite.size else -100.0
    thr = max(floor + 12.0, -55.0)
    return 1.0 / (1.0 + np.exp(-(db - thr) / 2.0))


def get_speech_timestamps(audio: np.ndarray, opts, model=None, sampling_rate: int = 16000, probs=None) -> List[dict]:
    threshold = opts.threshold
    neg = opts.neg_threshold if opts.neg_threshold is not None else max(threshold - 0.15, 0.01)
    min_speech = sampling_rate * opts.min_speech_duration_ms / 1000
    pad = sampling_rate * opts.speech_pad_ms / 1000
    max_speech = sampling_rate * opts.max_speech_duration_s - WINDOW - 2 * pad
    min_silence = sampling_rate * opts.min_silence_duration_ms / 1000
    min_silence_at_max = sampling_rate * 98 / 1000
    n = len(audio)
    if probs is None:
        probs = speech_probs(audio, model)
    triggered = False
    speeches: List[dict] = []
    cur: dict = {}
    temp_end = prev_end = next_start = 0
    for i, p in enumerate(probs):
        pos = WINDOW * i
        if p >= threshold and temp_end:
            temp_end = 0
            if next_start < prev_end:
                next_start = pos
        if p >= threshold and not triggered:
            triggered = True
            cur["start"] = pos
            continue
        if triggered and pos - cur["start"] > max_speech:
            if prev_end:
                cur["end"] = prev_end
                speeches.append(cur)
                cur = {}
                if next_start < prev_end:
                    triggered = False
                else:
                    cur["start"] = next_start
                prev_end = next_start = temp_end = 0
            else:
                cur["end"] = pos
                speeches.append(cur)
                cur = {}
                prev_end = next_start = temp_end = 0
                triggered = False
                continue
        if p < neg and triggered:
            if not temp_end:
                temp_end = pos
            if pos - temp_end > min_silence_at_max:
                prev_end = temp_end
            if pos - temp_end < min_silence:
                continue
            cur["end"] = temp_end
            if cur["end"] - cur["start"] > min_speech:
                speeches.append(cur)
            cur = {}
            prev_end = next_start = temp_end = 0
            triggered = False
            continue
    if cur and n - cur["start"] > min_speech:
        cur["end"] = n
        speeches.append(cur)
    for i, sp in enumerate(speeches):
        if i == 0:
            sp["start"] = int(max(0, sp["start"] - pad))
        if i != len(speeches) - 1:
            gap = speeches[i + 1]["start"] - sp["end"]
            if gap < 2 * pad:
                sp["end"] += int(gap // 2)
                speeches[i + 1]["start"] = int(max(0, speeches[i + 1]["start"] - gap // 2))
            else:
                sp["end"] = int(min(n, sp["end"] + pad))
                speeches[i + 1]["start"] = int(max(0, speeches[i + 1]["start"] - pad))
        else:
            sp["end"] = int(min(n, sp["end"] + pad))
    return speeches


def collect_chunks(audio: np.ndarray, chunks: List[dict]) -> np.ndarray:
    if not chunks:
        return np.zeros(0, dtype=np.float32)
    return np.concatenate([audio[c["start"]: c["end"]] for c in chunks]).astype(np.float32)


class SpeechTimestampsMap:
    def __init__(self, chunks: List[dict], sampling_rate: int, time_precision: int = 2):
        self.sampling_rate = sampling_rate
        self.time_precision = time_precision
        self.chunk_end_sample: List[int] = []
        self.total_silence_before: List[float] = []
        prev_end = silent = 0
        for c in chunks:
            silent += c["start"] - prev_end
            prev_end = c["end"]
            self.chunk_end_sample.append(c["end"] - silent)
            self.total_silence_before.append(silent / sampling_rate)

    def get_chunk_index(self, time: float, is_end: bool = False) -> int:
        """faster-whisper 1.1: a segment END that falls exactly on a chunk's last sample stays in that chunk
        (a plain bisect would move it into the next chunk and add the following silence gap to it)."""
        sample = int(time * self.sampling_rate)
        if is_end and sample in self.chunk_end_sample:
            return self.chunk_end_sample.index(sample)
        return min(bisect.bisect(self.chunk_end_sample, sample), len(self.chunk_end_sample) - 1)

    def get_original_time(self, time: float, chunk_index=None, is_end: bool = False) -> float:
        if chunk_index is None:
            chunk_index = self.get_chunk_index(time, is_end)
        return round(self.total_silence_before[chunk_index] + time, self.time_precision)


def restore_speech_timestamps(segments: Iterable, chunks: List[dict], sampling_rate: int):
    m = SpeechTimestampsMap(chunks, sampling_rate)
    for seg in segments:
        if seg.words:
            words = []
            for w in seg.words:
                ci = m.get_chunk_index((w.start + w.end) / 2)
                w.start = m.get_original_time(w.start, ci)
                w.end = m.get_original_time(w.end, ci)
                words.append(w)
            seg.start, seg.end, seg.words = words[0].start, words[-1].end, words
        else:
            seg.start = m.get_original_time(seg.start)
            seg.end = m.get_original_time(seg.end, is_end=True)
        yield seg
