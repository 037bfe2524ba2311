"""Multi-file window batching: BatchedInferencePipeline.transcribe_many packs the windows
of several files into shared decode batches.  Each file's result must be what transcribe() gives for that file
alone: the same windows, tokens and segment times (relative to the file).  With word timestamps the batched
alignment's DTW meets near-ties on the random-weight model that depend on the alignment batch's composition
(tests/test_gpu_words.py measures the same effect), so word times are compared with a tolerance."""
import numpy as np
import pytest

from vlog_amd.audio import speech_like

pytestmark = pytest.mark.gpu


def _files():
    gap = np.zeros(16000 * 4, np.float32)
    return [np.concatenate([speech_like(25.0, 1200), gap, speech_like(18.0, 1201)]),
            speech_like(21.0, 1202),
            np.concatenate([speech_like(40.0, 1203), gap, speech_like(33.0, 1204)])]


def _key(segs):
    return [(s.tokens, s.start, s.end) for s in segs]


@pytest.mark.parametrize("vad,words", [(False, False), (True, True)])
def test_transcribe_many_equals_per_file(vad, words):
    from vlog_amd.transcribe import BatchedInferencePipeline, WhisperModel
    model = WhisperModel("synthetic:tiny:3", device="cuda", eot_after=60)
    pipe = BatchedInferencePipeline(model, max_batch_windows=4)       # several mixed batches
    files = _files()
    kw = dict(language="en", beam_size=1, temperature=0.0, without_timestamps=False, vad_filter=vad,
              word_timestamps=words)
    many = pipe.transcribe_many(files, **kw)
    assert len(many) == len(files)
    for x, (segs, info) in zip(files, many):
        ref, rinfo = pipe.transcribe(x, **kw)
        ref = list(ref)
        assert info.duration == rinfo.duration and info.duration_after_vad == rinfo.duration_after_vad
        assert [s.tokens for s in segs] == [s.tokens for s in ref]
        if not words:
            assert _key(segs) == _key(ref)
            continue
        wa = [(w.word, w.start, w.end) for s in segs for w in s.words]
        wb = [(w.word, w.start, w.end) for s in ref for w in s.words]
        assert [w[0] for w in wa] == [w[0] for w in wb]
        close = np.mean([abs(a[1] - b[1]) <= 0.1 and abs(a[2] - b[2]) <= 0.1 for a, b in zip(wa, wb)]) if wa else 1.0
        assert close >= 0.8, close
        seg_close = np.mean([abs(a.start - b.start) <= 0.1 and abs(a.end - b.end) <= 0.1 for a, b in zip(segs, ref)])
        assert seg_close >= 0.8, seg_close
