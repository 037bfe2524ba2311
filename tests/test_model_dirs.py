"""CPU: local model directories (no downloads): HF safetensors and CTranslate2 model.bin readers, and a local
tokenizer.json, on builder-written fixtures (tests/model_fixtures.py) with seeded synthetic weights.  The
CTranslate2 reader is pinned only by this fixture writer (CTranslate2 is not installed here): parity unpinned
against real CTranslate2 files."""
import numpy as np
import pytest
import torch

from tests.model_fixtures import write_ct2_dir, write_hf_dir, write_tokenizer_json
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import resolve_model, synthetic_state_dict


@pytest.fixture(scope="module")
def tiny():
    dims = model_dims("tiny")
    return dims, synthetic_state_dict(dims, seed=3, eot_after=60)


def test_hf_dir_roundtrip(tiny, tmp_path):
    dims, sd = tiny
    write_hf_dir(str(tmp_path), sd, dims)
    d2, sd2, mdir = resolve_model(str(tmp_path))
    assert mdir == str(tmp_path)
    assert (d2.n_mels, d2.n_state, d2.n_head, d2.n_enc_layer, d2.n_dec_layer, d2.n_vocab) == \
           (dims.n_mels, dims.n_state, dims.n_head, dims.n_enc_layer, dims.n_dec_layer, dims.n_vocab)
    assert set(sd2) == set(sd)
    for k in sd:
        assert torch.equal(sd2[k], sd[k]), k


@pytest.mark.parametrize("dtype,tol", [("float32", 0.0), ("float16", 1e-3), ("bfloat16", 8e-3), ("int8", 1.0 / 127)])
def test_ct2_dir_roundtrip(tiny, tmp_path, dtype, tol):
    dims, sd = tiny
    write_ct2_dir(str(tmp_path), sd, dims, dtype)
    d2, sd2, mdir = resolve_model(str(tmp_path))
    assert (d2.n_mels, d2.n_state, d2.n_head, d2.n_enc_layer, d2.n_dec_layer, d2.n_vocab) == \
           (dims.n_mels, dims.n_state, dims.n_head, dims.n_enc_layer, dims.n_dec_layer, dims.n_vocab)
    assert d2.alignment_heads == tuple(tuple(h) for h in dims.default_alignment_heads())
    assert set(sd2) == set(sd)
    for k in sd:
        a, b = sd[k].numpy(), sd2[k].numpy()
        assert a.shape == b.shape, k
        if k.endswith(".weight") and a.ndim == 2:
            rowmax = np.abs(a).max(axis=1, keepdims=True)
            # int8: half a quantisation step of the row's scale; fp16/bf16: relative rounding (+ fp16 subnormals)
            assert np.all(np.abs(a - b) <= tol * np.maximum(np.abs(a), rowmax if dtype == "int8" else 0) + 1e-7), k
        else:
            assert np.array_equal(a, b), k                # biases, norms, positions, conv kernels stay float32


def test_ct2_reader_rejects_other_models(tiny, tmp_path):
    import struct
    with open(tmp_path / "model.bin", "wb") as f:
        f.write(struct.pack("<I", 6))
        b = b"TransformerSpec"
        f.write(struct.pack("<H", len(b) + 1) + b + b"\0")
        f.write(struct.pack("<II", 1, 0))
        f.write(struct.pack("<I", 0))
    with pytest.raises(ValueError, match="not Whisper"):
        resolve_model(str(tmp_path))


def test_tokenizer_json_layout_and_decode(tiny, tmp_path):
    from tokenizers import Tokenizer as HFTok
    dims, _ = tiny
    write_tokenizer_json(str(tmp_path), dims)
    path = str(tmp_path / "tokenizer.json")
    tok = Tokenizer(dims, language="en", tokenizer_json=path)
    st = dims.specials
    assert tok.sot_sequence == [st.sot, st.lang_token("en"), st.transcribe]
    hf = HFTok.from_file(path)
    ids = [220, 300, 1000, 40000, st.eot, st.timestamp_begin + 5, 7000]
    assert tok.decode(ids) == hf.decode([i for i in ids if i < st.eot], skip_special_tokens=True)
    assert tok.decode_with_timestamps(ids).count("<|0.10|>") == 1
    assert tok.encode(tok.decode([300, 1000])) == [300, 1000] or tok.decode(tok.encode(tok.decode([300, 1000]))) == tok.decode([300, 1000])
