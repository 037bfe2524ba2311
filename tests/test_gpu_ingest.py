"""Streaming ingest (vlog_amd/ingest.py): s16le PCM read from a pipe fed by a simulated
ffmpeg (a producer thread writing ragged chunks, odd byte counts included) -> pinned staging -> device ->
log-mel computed while the stream is open.  The PCM and the finalised features must be bit-identical to the
one-shot path on the same samples, and the throughput pipeline must give the same transcript from either."""
import os
import threading

import numpy as np
import pytest
import torch

from vlog_amd.audio import speech_like

pytestmark = pytest.mark.gpu


def _producer(fd, data: bytes, seed: int):
    rng = np.random.default_rng(seed)
    o = 0
    with os.fdopen(fd, "wb", buffering=0) as w:
        while o < len(data):
            n = int(rng.integers(1, 70000))
            w.write(data[o: o + n])
            o += n


def _ingest(eng, pcm_i16: np.ndarray, seed: int = 0, staging: int = 1 << 16):
    from vlog_amd.ingest import StreamingIngest
    r, w = os.pipe()
    t = threading.Thread(target=_producer, args=(w, pcm_i16.astype("<i2").tobytes(), seed))
    t.start()
    ing = StreamingIngest(eng, staging_samples=staging, initial_capacity=16000)
    with os.fdopen(r, "rb", buffering=0) as f:
        while True:
            b = f.read(int(np.random.default_rng(seed + 1).integers(1000, 50000)))
            if not b:
                break
            ing.feed(b)
    t.join()
    return ing.finish()


@pytest.fixture(scope="module")
def model():
    from vlog_amd.transcribe import WhisperModel
    return WhisperModel("synthetic:tiny:3", device="cuda", eot_after=60)


@pytest.mark.parametrize("seconds", [61.3, 0.0125, 0.5])
def test_streamed_features_bitexact(model, seconds):
    x = speech_like(max(seconds, 0.001), 77)[: int(seconds * 16000)]
    pcm = np.round(x * 32768).astype(np.int16)
    res = _ingest(model.engine, pcm, seed=int(seconds * 10))
    ref_pcm = torch.from_numpy(pcm.astype(np.float32) / 32768.0)
    assert res.n_samples == pcm.size
    assert torch.equal(res.pcm.cpu(), ref_pcm)
    ref = model.engine.features(ref_pcm.cuda())
    assert res.features.shape == ref.shape
    assert torch.equal(res.features, ref)


def test_pipeline_from_stream_equals_array(model):
    from vlog_amd.transcribe import BatchedInferencePipeline
    x = np.concatenate([speech_like(40.0, 81), np.zeros(16000 * 5, np.float32), speech_like(25.0, 82)])
    pcm = np.round(x * 32768).astype(np.int16)
    res = _ingest(model.engine, pcm, seed=3)
    pipe = BatchedInferencePipeline(model, max_batch_windows=8)
    kw = dict(language="en", beam_size=1, temperature=0.0, without_timestamps=False, vad_filter=True)
    a, ia = pipe.transcribe(res, **kw)
    b, ib = pipe.transcribe(pcm.astype(np.float32) / 32768.0, **kw)
    assert [(s.tokens, s.start, s.end) for s in a] == [(s.tokens, s.start, s.end) for s in b]
    assert ia.duration == ib.duration and ia.duration_after_vad == ib.duration_after_vad
