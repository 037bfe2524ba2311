"""End-to-end transcription restatement on the CPU oracle (TEST INFRASTRUCTURE ONLY).

faster-whisper 1.1.x `WhisperModel.transcribe` -> `generate_segments` -> `generate_with_fallback` [FW↑],
the call the reference worker makes (`worker/transcription.py:105-111`), restated independently of the
product's host code (vlog_amd/transcribe.py) so tests can compare the two end to end:
seek loop over 30 s windows, <|startofprev|> prompt of the last 223 tokens, temperature fallback on
compression ratio / avg log-prob with the no-speech exemption, skip on no_speech_prob, segment split at
timestamp pairs, optional word timestamps.  Sampling uses the engine's counter-based Gumbel noise
(oracle/decode.py gumbel_noise), keyed on (window index + temperature index, hypothesis, step, token).
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


# ----------------------------------------------------------------------------------------------- word timestamps
# faster-whisper 1.1.x `find_alignment` / `add_word_timestamps` and openai `merge_punctuations` [FW↑], restated
# here independently of vlog_amd/transcribe.py so the product's host logic can be compared against it.

PREPEND = "\"'“¿([{-"
APPEND = "\"'.。,，!！?？:：”)]}、"
SENTENCE_END = ".。!！?？"


def words_from_alignment(tok, text_tokens, probs, text_idx, time_idx, tokens_per_second=50):
    """One window's alignment -> [dict(word, tokens, start, end, probability)] (find_alignment's tail)."""
    words, word_tokens = tok.split_to_word_tokens(list(text_tokens) + [tok.eot])
    if len(word_tokens) <= 1:
        return []
    bounds = [0]
    for wt in word_tokens[:-1]:
        bounds.append(bounds[-1] + len(wt))
    if len(bounds) <= 1:
        return []
    text_idx, time_idx = np.asarray(text_idx), np.asarray(time_idx)
    is_jump = np.concatenate([[True], text_idx[1:] != text_idx[:-1]])
    jump_t = time_idx[is_jump] / tokens_per_second
    out = []
    for k in range(len(bounds) - 1):
        a, b = bounds[k], bounds[k + 1]
        out.append(dict(word=words[k], tokens=list(word_tokens[k]), start=jump_t[a], end=jump_t[b],
                        probability=np.mean(probs[a:b])))
    return out


def merge_punctuations(ws, prepended=PREPEND, appended=APPEND):
    """openai merge_punctuations on a word list (in place)."""
    j = len(ws) - 1
    for i in range(len(ws) - 2, -1, -1):
        a, b = ws[i], ws[j]
        if a["word"].startswith(" ") and a["word"].strip() in prepended:
            b["word"], b["tokens"] = a["word"] + b["word"], a["tokens"] + b["tokens"]
            a["word"], a["tokens"] = "", []
        else:
            j = i
    i = 0
    for j in range(1, len(ws)):
        a, b = ws[i], ws[j]
        if not a["word"].endswith(" ") and b["word"] in appended:
            a["word"], a["tokens"] = a["word"] + b["word"], a["tokens"] + b["tokens"]
            b["word"], b["tokens"] = "", []
        else:
            i = j


def add_word_timestamps(groups, tok, alignments, last_speech, prepended=PREPEND, appended=APPEND):
    """groups: per window, its split segments (dicts with seek/start/end/tokens; modified in place: start/end
    adjusted, `words` added); alignments: per window, words_from_alignment(...) of all its text tokens.
    -> the new last speech timestamp."""
    stats = []
    for al in alignments:
        d = np.array([w["end"] - w["start"] for w in al])
        d = d[d.nonzero()]
        med = min(0.7, float(np.median(d))) if len(d) else 0.0
        mx = 2 * med
        if len(d):
            for i in range(1, len(al)):
                if al[i]["end"] - al[i]["start"] > mx:
                    if al[i]["word"] in SENTENCE_END:
                        al[i]["end"] = al[i]["start"] + mx
                    elif al[i - 1]["word"] in SENTENCE_END:
                        al[i]["start"] = al[i]["end"] - mx
        merge_punctuations(al, prepended, appended)
        stats.append((med, mx))
    for g, segs_ in enumerate(groups):
        al, (med, mx) = alignments[g], stats[g]
        off = segs_[0]["seek"] / 100.0
        wi = 0
        for sub in segs_:
            need = len([t for t in sub["tokens"] if t < tok.eot])
            got, words = 0, []
            while wi < len(al) and got < need:
                w = al[wi]
                if w["word"]:
                    words.append(dict(word=w["word"], start=round(off + w["start"], 2), end=round(off + w["end"], 2),
                                      probability=w["probability"]))
                got += len(w["tokens"])
                wi += 1
            if words:
                w0 = words[0]
                if w0["end"] - last_speech > 4 * med and (
                        w0["end"] - w0["start"] > mx or (len(words) > 1 and words[1]["end"] - w0["start"] > 2 * mx)):
                    if len(words) > 1 and words[1]["end"] - words[1]["start"] > mx:
                        cut = max(words[1]["end"] / 2, words[1]["end"] - mx)
                        w0["end"] = words[1]["start"] = cut
                    w0["start"] = max(0, w0["end"] - mx)
                if sub["start"] < w0["end"] and sub["start"] - 0.5 > w0["start"]:
                    w0["start"] = max(0, min(w0["end"] - med, sub["start"]))
                else:
                    sub["start"] = w0["start"]
                wl = words[-1]
                if sub["end"] > wl["start"] and sub["end"] + 0.5 < wl["end"]:
                    wl["end"] = max(wl["start"] + med, sub["end"])
                else:
                    sub["end"] = wl["end"]
                last_speech = sub["end"]
            sub["words"] = words
    return last_speech


def last_word_end(segs_):
    for s in reversed(segs_):
        for w in reversed(s.get("words") or []):
            return w["end"]
    return segs_[-1]["end"] if segs_ else None


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

    def align(self, cross, sot_sequence, text_tokens, num_frames):
        dims = self.model.dims
        return find_alignment(self.model, cross, sot_sequence, text_tokens, dims.specials, num_frames,
                              dims.default_alignment_heads())


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
    last_speech = 0.0
    window = 0                                  # seeds: window index + temperature index (vlog_amd seeding)
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
                                  sampling_temperature=T, num_hypotheses=5 if T > 0 else 1, seed=window + i)
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
        window += 1
        if res.no_speech_prob > 0.6 and not alp > -1.0:
            seek += size
            continue
        cur, seek, single = _split(res.tokens, st.timestamp_begin, toff, size, dur, seek)
        if word_timestamps:
            text_tokens = [t for s in cur for t in s["tokens"] if t < st.eot]
            al = []
            if text_tokens:
                probs, ti, tj = be.align(cross, tok.sot_sequence, text_tokens, size)
                al = words_from_alignment(tok, text_tokens, probs, ti, tj)
            last_speech = add_word_timestamps([cur], tok, [al], last_speech)
            if not single:
                lw = last_word_end(cur)
                if lw is not None and lw > toff:
                    seek = round(lw * 100)
        for s in cur:
            text = tok.decode(s["tokens"])
            if s["start"] == s["end"] or not text.strip():
                continue
            all_tokens.extend(s["tokens"])
            out.append(dict(start=s["start"], end=s["end"], text=text, tokens=s["tokens"], avg_logprob=alp,
                            no_speech_prob=res.no_speech_prob, temperature=T, words=s.get("words")))
        if not condition_on_previous_text or T > 0.5:
            reset_since = len(all_tokens)
    return out, language
