"""Whisper tokenizer (host side).

Mirrors faster-whisper's `Tokenizer` [FW↑ 1.1.x] — the object behind `segment.text`, which the worker
reads (`worker/transcription.py:117-127`): `sot_sequence`, `decode` (text tokens only), `encode`,
`non_speech_tokens`, `split_to_word_tokens`, and the special-token properties.

Two vocabularies:
  * a local `tokenizer.json` (HF `tokenizers`, byte-level BPE) when the model directory has one;
  * otherwise a seeded *synthetic* byte-level vocabulary for synthetic weights: ids 0..255 are the 256
    bytes in GPT-2's byte order (so " " is id 220, the SuppressBlank token), ids 256..eot-1 are seeded
    pseudo-words, then the standard special tokens (vlog_amd/dims.py).  Text produced from synthetic
    weights is arbitrary but deterministic, so both engines' transcripts can be compared word for word.
"""
from __future__ import annotations

import os
import string
from functools import cached_property
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .dims import LANGUAGES, ModelDims, SpecialTokens


def _gpt2_byte_order() -> List[int]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    rest = [b for b in range(256) if b not in bs]
    return bs + rest


def _special_texts(st: SpecialTokens, n_vocab: int) -> Dict[int, str]:
    out = {st.eot: "<|endoftext|>", st.sot: "<|startoftranscript|>", st.translate: "<|translate|>",
           st.transcribe: "<|transcribe|>", st.sot_lm: "<|startoflm|>", st.sot_prev: "<|startofprev|>",
           st.no_speech: "<|nospeech|>", st.no_timestamps: "<|notimestamps|>"}
    for i in range(st.translate - st.lang_begin):
        out[st.lang_begin + i] = f"<|{LANGUAGES[i]}|>" if i < len(LANGUAGES) else f"<|lang{i}|>"
    for i in range(st.timestamp_begin, n_vocab):
        out[i] = f"<|{(i - st.timestamp_begin) * 0.02:.2f}|>"
    return out


class _SyntheticVocab:
    def __init__(self, st: SpecialTokens, n_vocab: int, seed: int = 0):
        self.st = st
        order = _gpt2_byte_order()
        self.pieces: List[bytes] = [bytes([b]) for b in order]
        rng = np.random.default_rng(seed + 7919)
        cons = list("bcdfghjklmnprstvwz") + ["th", "sh", "ch", "st", "tr", "br"]
        vows = list("aeiou") + ["ea", "ou", "ai"]
        while len(self.pieces) < st.eot:
            n_syl = int(rng.integers(1, 4))
            w = "".join(cons[rng.integers(len(cons))] + vows[rng.integers(len(vows))] for _ in range(n_syl))
            if rng.random() < 0.3:
                w += cons[rng.integers(len(cons))]
            if rng.random() < 0.1:
                w = w.capitalize()
            if rng.random() < 0.7:
                w = " " + w
            r = rng.random()
            if r < 0.03:
                w += "."
            elif r < 0.05:
                w += ","
            self.pieces.append(w.encode())
        self.special = _special_texts(st, n_vocab)
        self.lookup: Dict[bytes, int] = {}
        for i, p in enumerate(self.pieces):
            self.lookup.setdefault(p, i)
        self.maxlen = max(len(p) for p in self.pieces)

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        out = bytearray()
        text = []
        for t in ids:
            t = int(t)
            if t < len(self.pieces):
                out += self.pieces[t]
            elif not skip_special:
                text.append(out.decode("utf-8", errors="replace")); out = bytearray()
                text.append(self.special.get(t, ""))
        text.append(out.decode("utf-8", errors="replace"))
        return "".join(text)

    def encode(self, s: str) -> List[int]:
        b = s.encode()
        i, ids = 0, []
        while i < len(b):
            for L in range(min(self.maxlen, len(b) - i), 0, -1):
                t = self.lookup.get(b[i: i + L])
                if t is not None:
                    ids.append(t); i += L
                    break
        return ids


class _HFVocab:
    def __init__(self, path: str):
        from tokenizers import Tokenizer as HFTok
        self.tok = HFTok.from_file(path)

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        return self.tok.decode([int(t) for t in ids], skip_special_tokens=skip_special)

    def encode(self, s: str) -> List[int]:
        return self.tok.encode(s, add_special_tokens=False).ids

    def token_to_id(self, s: str) -> Optional[int]:
        return self.tok.token_to_id(s)


# Vocabularies are immutable once built and cost a model's worth of work to build (the synthetic one: 0.3 s of
# seeded word generation; a tokenizer.json: a file parse), while faster-whisper builds a Tokenizer per transcribe
# call around a tokenizer it loaded once.  So they are built once per process and shared.
_VOCABS: Dict[tuple, object] = {}


def _vocab_for(st: SpecialTokens, n_vocab: int, tokenizer_json: Optional[str], seed: int):
    if tokenizer_json and os.path.isfile(tokenizer_json):
        path = os.path.abspath(tokenizer_json)
        key = ("json", path, os.path.getmtime(path))
        if key not in _VOCABS:
            _VOCABS[key] = _HFVocab(path)
    else:
        key = ("synthetic", n_vocab, st.eot, st.sot, st.lang_begin, st.timestamp_begin, seed)
        if key not in _VOCABS:
            _VOCABS[key] = _SyntheticVocab(st, n_vocab, seed)
    return _VOCABS[key]


class Tokenizer:
    """faster-whisper-shaped tokenizer: Tokenizer(vocab, multilingual, task, language)."""

    def __init__(self, dims: ModelDims, task: Optional[str] = "transcribe", language: Optional[str] = None,
                 tokenizer_json: Optional[str] = None, seed: int = 0):
        self.dims = dims
        self.st = dims.specials
        self.multilingual = dims.multilingual
        self.vocab = _vocab_for(self.st, dims.n_vocab, tokenizer_json, seed)
        if isinstance(self.vocab, _HFVocab):
            sot = self.vocab.token_to_id("<|startoftranscript|>")
            if sot is not None and sot != self.st.sot:
                raise ValueError(f"tokenizer.json <|startoftranscript|>={sot} does not match the model layout")
        self.task = self.transcribe if task == "transcribe" else self.translate if task == "translate" else None
        self.language_code = language or "en"
        self.language = self.st.lang_token(self.language_code) if (self.multilingual and language) else None

    # -------- special tokens (faster-whisper Tokenizer properties)
    @property
    def eot(self): return self.st.eot
    @property
    def sot(self): return self.st.sot
    @property
    def transcribe(self): return self.st.transcribe
    @property
    def translate(self): return self.st.translate
    @property
    def sot_lm(self): return self.st.sot_lm
    @property
    def sot_prev(self): return self.st.sot_prev
    @property
    def no_speech(self): return self.st.no_speech
    @property
    def no_timestamps(self): return self.st.no_timestamps
    @property
    def timestamp_begin(self): return self.st.timestamp_begin

    @property
    def sot_sequence(self) -> List[int]:
        seq = [self.sot]
        if self.language is not None:
            seq.append(self.language)
        if self.task is not None and self.multilingual:
            seq.append(self.task)
        return seq

    def encode(self, text: str) -> List[int]:
        return self.vocab.encode(text)

    def decode(self, tokens: Sequence[int]) -> str:
        return self.vocab.decode([t for t in tokens if t < self.eot])

    def decode_with_timestamps(self, tokens: Sequence[int]) -> str:
        return self.vocab.decode(tokens, skip_special=False)

    @cached_property
    def non_speech_tokens(self) -> Tuple[int, ...]:
        symbols = list('"#()*+/:;<=>@[\\]^_`{|}~「」『』')
        symbols += "<< >> <<< >>> -- --- -( -[ (' (\" (( )) ((( ))) [[ ]] {{ }} ♪♪ ♪♪♪".split()
        misc = set("♩♪♫♬♭♮♯")
        result = set()
        for s in (" -", " '"):
            e = self.encode(s)
            if e:
                result.add(e[0])
        for sym in symbols + list(misc):
            for toks in (self.encode(sym), self.encode(" " + sym)):
                if toks and (len(toks) == 1 or sym in misc):
                    result.add(toks[0])
        return tuple(sorted(result))

    def suppressed_tokens(self, suppress_tokens: Optional[Sequence[int]] = (-1,)) -> Tuple[int, ...]:
        """faster-whisper `get_suppressed_tokens`."""
        s = list(suppress_tokens or [])
        if -1 in s:
            s = [t for t in s if t >= 0] + list(self.non_speech_tokens)
        s += [self.transcribe, self.translate, self.sot, self.sot_prev, self.sot_lm]
        return tuple(sorted(set(s)))

    # -------- word splitting (word_timestamps)
    def split_to_word_tokens(self, tokens: List[int]) -> Tuple[List[str], List[List[int]]]:
        if self.language_code in {"zh", "ja", "th", "lo", "my", "yue"}:
            return self.split_tokens_on_unicode(tokens)
        return self.split_tokens_on_spaces(tokens)

    def _decode_one(self, t: int) -> str:
        """decode_with_timestamps([t]), memoised on the (shared, immutable) vocabulary: word splitting decodes most
        tokens alone, once per word."""
        memo = self.vocab.__dict__.setdefault("_one", {})
        s = memo.get(t)
        if s is None:
            s = memo[t] = self.decode_with_timestamps([t])
        return s

    def split_tokens_on_unicode(self, tokens: List[int]):
        full = self.decode_with_timestamps(tokens)
        rep = "�"
        words, word_tokens, cur = [], [], []
        off = 0
        for t in tokens:
            cur.append(t)
            dec = self._decode_one(int(t)) if len(cur) == 1 else self.decode_with_timestamps(cur)
            idx = dec.find(rep)
            idx = None if idx < 0 else idx + off
            if idx is None or (idx < len(full) and full[idx] == rep):
                words.append(dec); word_tokens.append(cur); cur = []; off += len(dec)
        return words, word_tokens

    def split_tokens_on_spaces(self, tokens: List[int]):
        subwords, subtoks = self.split_tokens_on_unicode(tokens)
        words, word_tokens = [], []
        for sw, st in zip(subwords, subtoks):
            special = st[0] >= self.eot
            with_space = sw.startswith(" ")
            punct = sw.strip() in string.punctuation
            if special or with_space or punct or not words:
                words.append(sw); word_tokens.append(list(st))
            else:
                words[-1] += sw; word_tokens[-1].extend(st)
        return words, word_tokens
