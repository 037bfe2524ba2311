"""Failure contract: numeric breakage detected on the device fails the call with an
error instead of decoding into garbage tokens.  The worker turns any exception from `transcribe` into the job's
FAILED status (reference worker/transcription.py:436-443).

The test-only engine option `debug_nan_row` overwrites one logits row with NaN before every token selection of
wm_generate (engine.cpp debug_nan); the selection kernel finds the non-finite row (search.hip), records it in the
device error word, and the host raises at its next poll."""
import numpy as np
import pytest
import torch

from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiny():
    from vlog_amd.engine import GpuEngine
    from vlog_amd.tokenizer import Tokenizer
    dims = model_dims("tiny")
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=3, eot_after=40), 0)
    W = 4
    x = np.concatenate([speech_like(30.0, 300 + i) for i in range(W)])
    mel = eng.features(torch.from_numpy(x))
    enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W)
    eng.reserve(W, W * 5)
    eng.cross_kv(enc, 0)
    tok = Tokenizer(dims, language="en")
    return eng, list(tok.sot_sequence), list(tok.suppressed_tokens([-1])), W


CASES = [dict(), dict(beam_size=5), dict(max_rows=2, compact=True), dict(temperature=0.7, num_hypotheses=3),
         dict(record_logprobs=True)]


@pytest.mark.parametrize("kw", CASES, ids=["greedy", "beam5", "row_set", "sampling_best_of3", "records"])
def test_nan_logits_row_raises(tiny, kw):
    eng, prompt, sup, W = tiny
    ok, _ = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=100, **kw)
    assert all(0 < len(r.tokens) < 100 for r in ok)
    eng.set_option("debug_nan_row", 1)
    try:
        assert eng.option("debug_nan_row") == 1
        with pytest.raises(RuntimeError, match="non-finite"):
            eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=100, **kw)
    finally:
        eng.set_option("debug_nan_row", -1)
    # the engine is usable after the failure, and decodes the same as before it
    again, _ = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=100, **kw)
    if not kw.get("temperature"):
        assert [r.tokens for r in again] == [r.tokens for r in ok]


def test_nan_whole_beam_group_ends_cleanly(tiny):
    """every hypothesis of one window non-finite -> beam_select sees no live candidate (nlive 0).
    The dead beams must take a valid lineage and token (not uninitialised LDS), the call raises with the error word,
    and the engine decodes the same afterwards."""
    eng, prompt, sup, W = tiny
    kw = dict(beam_size=5)
    ok, _ = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=100, **kw)
    eng.set_option("debug_nan_row", 5)          # window 1's five hypotheses
    eng.set_option("debug_nan_count", 5)
    try:
        assert eng.option("debug_nan_count") == 5
        with pytest.raises(RuntimeError, match="non-finite"):
            eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=100, **kw)
    finally:
        eng.set_option("debug_nan_row", -1)
        eng.set_option("debug_nan_count", 1)
    again, _ = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=100, **kw)
    assert [r.tokens for r in again] == [r.tokens for r in ok]


def test_bad_prompt_token_raises(tiny):
    eng, prompt, sup, W = tiny
    with pytest.raises(RuntimeError, match="vocabulary"):
        eng.generate([0], [[prompt[0], 10 ** 6]], suppress_tokens=sup, max_length=50)


def test_transcribe_raises_runtime_error(tmp_path):
    """The worker's call (beam 5, the sequential seek loop) raises RuntimeError when the device sees a NaN row."""
    from vlog_amd.audio import write_wav
    from vlog_amd.transcribe import WhisperModel
    model = WhisperModel("synthetic:tiny.en:0:margin", device="cpu", compute_type="int8")
    wav = tmp_path / "clip.wav"
    write_wav(str(wav), speech_like(30.0, 77))
    segs, _ = model.transcribe(str(wav), beam_size=5, temperature=0.0)
    assert len(list(segs)) >= 1
    model.engine.set_option("debug_nan_row", 0)
    try:
        with pytest.raises(RuntimeError, match="non-finite"):
            segs, _ = model.transcribe(str(wav), beam_size=5, temperature=0.0)
            list(segs)
    finally:
        model.engine.set_option("debug_nan_row", -1)
