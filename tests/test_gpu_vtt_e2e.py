"""Config 1 end to end: tiny.en (English-only vocabulary 51864, no language token), a 60 s clip -> WebVTT, the
way the worker calls it (`worker/transcription.py:81-85, 105-131, 377`), compared with the CPU oracle's host loop.

  * VTT bytes: the product's faster-whisper loop vs oracle/transcribe.py's independent restatement of that
    loop on the SAME decoder (GPU backend) -> byte-identical captions.
  * Full CPU oracle (encoder + decoder in the engine's numeric format, oracle host loop) vs the GPU: WER of
    the GPU transcript against the oracle transcript, and identical cue structure when the tokens agree.
"""
import numpy as np
import pytest
import torch

from oracle import transcribe as otr
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like, write_wav
from vlog_amd.metrics import word_error_rate
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.vtt import generate_webvtt
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu


class _Dims:
    def __init__(self, dims):
        self.dims = dims


class _GpuBackend:
    def __init__(self, model):
        self.m = model

    def encode(self, window):
        enc = self.m.engine.encode(torch.from_numpy(np.ascontiguousarray(window, dtype=np.float32)).cuda(), [0], [3000])
        self.m.engine.cross_kv(enc, 0)
        return 0

    def generate(self, slot, prompt, opt):
        from oracle.decode import GenerateResult
        st = self.m.dims.specials
        res, _ = self.m.engine.generate([slot], [prompt], beam_size=opt.beam_size, patience=opt.patience,
                                        length_penalty=opt.length_penalty, max_length=opt.max_length,
                                        suppress_tokens=opt.suppress_tokens, suppress_blank=opt.suppress_blank,
                                        max_initial_timestamp_index=opt.max_initial_timestamp_index,
                                        sot_index=prompt.index(st.sot))
        r = res[0]
        return GenerateResult(r.tokens, r.score, r.no_speech_prob, r.cum_logprob)

    def detect_language(self, slot):
        raise AssertionError("tiny.en is English-only: no language detection")


@pytest.fixture(scope="module")
def tiny_en(tmp_path_factory):
    from vlog_amd.transcribe import WhisperModel
    model = WhisperModel("synthetic:tiny.en:3", device="cpu", compute_type="int8", eot_after=60)   # worker's args
    x = np.concatenate([speech_like(30.0, 900), speech_like(30.0, 901)])                          # 60 s clip
    wav = tmp_path_factory.mktemp("cfg1") / "clip.wav"
    write_wav(str(wav), x)
    return model, str(wav)


def _vtt(segs):
    return generate_webvtt([{"start": s["start"], "end": s["end"], "text": s["text"]} for s in segs])


def test_tiny_en_vtt_bytes_match_oracle_host_loop(tiny_en):
    from vlog_amd.audio import load_audio
    model, wav = tiny_en
    assert not model.is_multilingual and model.dims.n_vocab == 51864
    segs, info = model.transcribe(wav, language=None, task="transcribe", beam_size=5, temperature=0.0)
    segs = [dict(start=s.start, end=s.end, text=s.text, tokens=s.tokens) for s in segs]
    assert info.language == "en" and segs
    pcm = load_audio(wav)
    feats = model.engine.features(torch.from_numpy(pcm)).cpu().numpy()
    ref, lang = otr.transcribe(_Dims(model.dims), lambda l: Tokenizer(model.dims, language=l), pcm, beam_size=5,
                               temperatures=(0.0,), features=feats, backend=_GpuBackend(model))
    assert lang is None or lang == "en"
    assert [s["tokens"] for s in segs] == [r["tokens"] for r in ref]
    vtt, vtt_ref = _vtt(segs), _vtt(ref)
    assert vtt == vtt_ref
    assert vtt.startswith("WEBVTT\n\n") and vtt.count(" --> ") == len(segs)


def test_tiny_en_vs_cpu_oracle_transcript(tiny_en):
    """The whole path on the CPU oracle (log-mel, encoder and decoder in the engine's numeric format, oracle
    seek loop) vs the GPU path on the same WAV."""
    from vlog_amd.audio import load_audio
    import json, os
    model, wav = tiny_en
    sd = synthetic_state_dict(model.dims, seed=3, eot_after=60)
    orc = OracleWhisper(round_bf16(sd), model.dims, np.float32, bf16_acts=True, bf16_enc=True)
    pcm = load_audio(wav)
    ref, _ = otr.transcribe(orc, lambda l: Tokenizer(model.dims, language=l), pcm, beam_size=5, temperatures=(0.0,))
    segs, _ = model.transcribe(wav, language=None, beam_size=5, temperature=0.0)
    segs = list(segs)
    hyp_text = " ".join(s.text.strip() for s in segs)
    ref_text = " ".join(r["text"].strip() for r in ref)
    wer = word_error_rate(ref_text, hyp_text)
    same = [s.tokens for s in segs] == [r["tokens"] for r in ref]
    p = os.environ.get("VLOG_AMD_PARITY_OUT")
    if p:
        with open(p, "a") as f:
            f.write(json.dumps({"name": "tiny.en 60 s vs CPU oracle", "wer": wer, "tokens_identical": same,
                                "segments": len(segs), "segments_oracle": len(ref)}) + "\n")
    if same:
        assert _vtt([dict(start=s.start, end=s.end, text=s.text) for s in segs]) == _vtt(ref)
    assert wer <= 0.05, wer


def test_tiny_en_worker_call_with_vad(tiny_en):
    """The worker's literal call (vad_filter=True, default temperature fallback) through the compat overlay."""
    import os, sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "compat"))
    import faster_whisper
    model, wav = tiny_en
    assert faster_whisper.WhisperModel is type(model)
    segments, info = model.transcribe(wav, language=None, task="transcribe", beam_size=5, vad_filter=True)
    seg_list = [{"start": s.start, "end": s.end, "text": s.text} for s in segments]
    vtt = generate_webvtt(seg_list)
    assert info.language == "en" and vtt.startswith("WEBVTT\n\n") and vtt.count(" --> ") == len(seg_list)
    assert all(0.0 <= s["start"] <= s["end"] for s in seg_list)
