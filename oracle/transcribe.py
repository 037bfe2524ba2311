"""End-to-end transcription restatement on the CPU oracle (TEST INFRASTRUCTURE ONLY).

faster-whisper 1.1.x `WhisperModel.transcribe` -> `generate_segments` -> `generate_with_fallback` [FW↑],
the call the reference worker makes (`worker/transcription.py:105-111`), restated independently of the
product's host code (vlog_amd/transcribe.py) so tests can compare the two end to end:
seek loop over 30 s windows, <|startofprev|> prompt of the last 223 tokens, temperature fallback on
compression ratio / avg log-prob with the no-speech exemption, skip on no_speech_prob, segment split at
timestamp pairs, optional word timestamps.  Sampling temperatures use numpy's RNG, so only the T = 0
path is expected to match token for token.
"""
from __future__ import annotations

import zlib
from typing import List, Optional

import numpy as np

from . import mel as omel
from .align import find_alignment
from .decode import GenerateOptions, detect_language, generate_one


def _cr(text: str) -> float:
    b = text.encode("utf-8")
    return len(b) / len(zlib.compress(b)) if b else 0.0


def _split(tokens, tb, time_offset, segment_size, segment_duration, seek):
    out = []
    single = len(tokens) >= 2 and tokens[-2] < tb <= tokens[-1]
    cons = [i for i in range(len(tokens)) if i > 0 and tokens[i] >= tb and tokens[i - 1] >= tb]
    if cons:
        slices = list(cons) + ([len(tokens)] if single else [])
        last = 0
        for cur in slices:
            sl = tokens[last:cur]
            out.append(dict(seek=seek, start=time_offset + (sl[0] - tb) * 0.02, end=time_offset + (sl[-1] - tb) * 0.02,
                            tokens=sl))
            last = cur
        seek = seek + segment_size if single else seek + (tokens[last - 1] - tb) * 2
    else:
        dur = segment_duration
        ts = [t for t in tokens if t >= tb]
        if ts and ts[-1] != tb:
            dur = (ts[-1] - tb) * 0.02
        out.append(dict(seek=seek, start=time_offset, end=time_offset + dur, tokens=tokens))
        seek += segment_size
    return out, seek, single


class OracleBackend:
    """The oracle's own encoder + decoder for the loop below."""

    def __init__(self, model, encoder=None):
        self.model = model
        self.encoder = encoder or (lambda w: model.encode(w[None]))

    def encode(self, window):
        return self.model.cross_kv(self.encoder(window))

    def generate(self, cross, prompt, opt):
        return generate_one(self.model, cross, prompt, self.model.dims.specials, opt)

    def detect_language(self, cross):
        return detect_language(self.model, cross, self.model.dims.specials)


def transcribe(model, tokenizer, audio: np.ndarray, beam_size: int = 5, temperatures=(0.0, 0.2, 0.4, 0.6, 0.8, 1.0),
               condition_on_previous_text: bool = True, suppress_tokens: Optional[List[int]] = None,
               word_timestamps: bool = False, language: Optional[str] = None, encoder=None, features=None,
               backend=None):
    """`encoder(mel_window [n_mels, 3000]) -> [1, 1500, d]` overrides the oracle encoder so a test can compare
    two decoders + host loops on the SAME encoder output (the encode/generate boundary); `features` likewise
    overrides the log-mel (tested separately against oracle/mel.py); `backend` (encode / generate /
    detect_language) replaces the oracle model entirely, so the HOST loops can be compared on one decoder.
    -> (segments [dict(start, end, text, tokens, avg_logprob, no_speech_prob, temperature, words)], language)."""
    dims = model.dims
    st = dims.specials
    feats = omel.log_mel(audio, dims.n_mels) if features is None else np.asarray(features, dtype=np.float32)
    content = feats.shape[1] - 1
    be = backend or OracleBackend(model, encoder)
    if language is None and dims.multilingual:
        language = be.detect_language(be.encode(omel.pad_or_trim(feats[:, :3000])))[0][0]
    tok = tokenizer(language)
    sup = list(suppress_tokens) if suppress_tokens is not None else list(tok.suppressed_tokens([-1]))
    seek, all_tokens, reset_since, out = 0, [], 0, []
    while seek < content:
        size = min(3000, content - seek)
        dur = size * 0.01
        toff = seek * 0.01
        cross = be.encode(omel.pad_or_trim(feats[:, seek: seek + size]))
        prev = all_tokens[reset_since:]
        prompt = ([st.sot_prev] + prev[-223:] if prev else []) + tok.sot_sequence
        results, below = [], []
        r = None
        for i, T in enumerate(temperatures):
            opt = GenerateOptions(beam_size=beam_size if T == 0 else 1, patience=1.0, length_penalty=1.0, max_length=448,
                                  suppress_tokens=sup, suppress_blank=True, max_initial_timestamp_index=50,
                                  sampling_temperature=T, num_hypotheses=5 if T > 0 else 1, seed=i)
            res = be.generate(cross, prompt, opt)
            n = len(res.tokens)
            alp = res.score * n / (n + 1)
            text = tok.decode(res.tokens).strip()
            cr = _cr(text)
            r = (res, alp, T, cr)
            results.append(r)
            fb = False
            if cr > 2.4:
                fb = True
            else:
                below.append(r)
            if alp < -1.0:
                fb = True
            if res.no_speech_prob > 0.6 and alp < -1.0:
                fb = False
            if not fb:
                break
        else:
            best = max(below or results, key=lambda x: x[1])
            r = (best[0], best[1], T, best[3])
        res, alp, T, cr = r
        if res.no_speech_prob > 0.6 and not alp > -1.0:
            seek += size
            continue
        cur, seek, single = _split(res.tokens, st.timestamp_begin, toff, size, dur, seek)
        if word_timestamps:
            text_tokens = [t for s in cur for t in s["tokens"] if t < st.eot]
            if text_tokens:
                probs, ti, tj = find_alignment(model, cross, tok.sot_sequence, text_tokens, st, size,
                                               dims.default_alignment_heads())
                for s in cur:
                    s["alignment"] = (probs, ti, tj)
        for s in cur:
            text = tok.decode(s["tokens"])
            if s["start"] == s["end"] or not text.strip():
                continue
            all_tokens.extend(s["tokens"])
            out.append(dict(start=s["start"], end=s["end"], text=text, tokens=s["tokens"], avg_logprob=alp,
                            no_speech_prob=res.no_speech_prob, temperature=T))
        if not condition_on_previous_text or T > 0.5:
            reset_since = len(all_tokens)
    return out, language
