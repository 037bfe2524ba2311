"""WhisperModel(<local directory>) on the MI355X: an HF safetensors directory and a CTranslate2 model.bin
directory (the faster-whisper deployment layout the worker's WHISPER_MODEL resolves to; reference
config.py:263, worker/transcription.py:81-85), each with a local tokenizer.json.  With the weights of
`synthetic:tiny:3` the directory models must decode exactly the same tokens, and segment text must come from
the tokenizer.json vocabulary."""
import numpy as np
import pytest

from tests.model_fixtures import write_ct2_dir, write_hf_dir, write_tokenizer_json
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dirs(tmp_path_factory):
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=3, eot_after=60)
    hf = tmp_path_factory.mktemp("hf")
    write_hf_dir(str(hf), sd, dims)
    write_tokenizer_json(str(hf), dims)
    ct = tmp_path_factory.mktemp("ct2")
    write_ct2_dir(str(ct), sd, dims, "float32")
    write_tokenizer_json(str(ct), dims)
    c8 = tmp_path_factory.mktemp("ct2i8")
    write_ct2_dir(str(c8), sd, dims, "int8")
    return str(hf), str(ct), str(c8)


def _run(model, x):
    segs, info = model.transcribe(x, language="en", beam_size=5, temperature=0.0)
    return [s for s in segs], info


def test_directory_models_decode_like_synthetic(dirs):
    from tokenizers import Tokenizer as HFTok
    from vlog_amd.transcribe import WhisperModel
    hf, ct, _ = dirs
    x = np.concatenate([speech_like(30.0, 700), speech_like(17.0, 701)])
    ref, _ = _run(WhisperModel("synthetic:tiny:3", device="cpu", eot_after=60), x)
    tj = HFTok.from_file(hf + "/tokenizer.json")
    for path in (hf, ct):
        m = WhisperModel(path, device="cpu", compute_type="int8")
        assert m._tokenizer_json is not None
        segs, info = _run(m, x)
        assert [s.tokens for s in segs] == [r.tokens for r in ref]
        for s in segs:
            assert s.text == tj.decode([t for t in s.tokens if t < m.dims.specials.eot], skip_special_tokens=True)


def test_int8_ct2_directory_runs(dirs):
    """compute_type int8 as faster-whisper stores it: the weights are dequantised to bf16 at load."""
    from vlog_amd.transcribe import WhisperModel
    _, _, c8 = dirs
    m = WhisperModel(c8, device="cpu", compute_type="int8")
    segs, info = _run(m, np.concatenate([speech_like(30.0, 702)]))
    assert segs and all(0.0 <= s.start <= s.end for s in segs)
