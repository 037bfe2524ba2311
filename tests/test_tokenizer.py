"""Tokenizer surface (faster-whisper Tokenizer): special ids, sot_sequence, decode, suppression, word split."""
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer


def test_special_layout_and_sot_sequence():
    d = model_dims("large-v3")
    t = Tokenizer(d, language="de")
    assert (t.eot, t.sot, t.transcribe, t.no_timestamps, t.timestamp_begin) == (50257, 50258, 50360, 50364, 50365)
    assert t.sot_sequence == [50258, 50259 + 2, 50360]
    en = Tokenizer(model_dims("tiny.en"))
    assert en.sot_sequence == [50257] and en.timestamp_begin == 50363


def test_decode_and_blank():
    t = Tokenizer(model_dims("base"), language="en")
    assert t.encode(" ") == [220] and t.decode([220]) == " "
    assert t.decode([t.sot, 220, t.eot, t.timestamp_begin]) == " "
    s = t.decode([300, 301, 302])
    assert isinstance(s, str) and len(s) > 0


def test_suppressed_tokens_and_words():
    t = Tokenizer(model_dims("base"), language="en")
    sup = t.suppressed_tokens([-1])
    for x in (t.transcribe, t.translate, t.sot, t.sot_prev, t.sot_lm):
        assert x in sup
    assert t.encode('"')[0] in sup
    words, toks = t.split_to_word_tokens([300, 301, 302, 303, t.eot])
    assert sum(len(x) for x in toks) == 5 and words[-1] == "<|endoftext|>"
    assert "".join(words[:-1]) == t.decode([300, 301, 302, 303])
