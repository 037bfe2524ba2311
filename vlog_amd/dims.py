"""Whisper model dimensions and the special-token layout.

The transcription worker picks a model by name (`WHISPER_MODEL`, reference `config.py:263`, default
"medium") and hands it to `WhisperModel(...)` (`worker/transcription.py:81-85`).  This table gives the
architecture of every name the reference's settings accept (`api/settings_service.py:868-892`) plus
large-v3 (the BASELINE metric's model) and large-v3-turbo.

Special-token ids are *derived* from the vocabulary size and the multilingual flag, exactly the way the
upstream vocabularies are laid out: regular BPE tokens, then <|endoftext|>,
<|startoftranscript|>, the language tokens, <|translate|>, <|transcribe|>, <|startoflm|>, <|startofprev|>,
<|nospeech|>, <|notimestamps|> and 1501 timestamp tokens <|0.00|> ... <|30.00|>.  When a real
`tokenizer.json` is present the ids are read from it instead (vlog_amd/tokenizer.py) and checked against
this layout.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

# Language codes in vocabulary order (the order of the <|xx|> tokens).  The set equals the reference's
# WHISPER_LANGUAGES (`api/schemas.py:16-117`, 100 codes including "yue").
LANGUAGES: Tuple[str, ...] = (
    "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id",
    "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg",
    "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br",
    "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si", "km", "sn", "yo", "so",
    "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn", "mt",
    "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su", "yue",
)

N_TIMESTAMPS = 1501          # <|0.00|> ... <|30.00|>
TIME_PRECISION = 0.02        # seconds per timestamp token
SAMPLE_RATE = 16000
N_FFT = 400
HOP_LENGTH = 160
CHUNK_LENGTH = 30
N_SAMPLES = CHUNK_LENGTH * SAMPLE_RATE       # 480000 samples per window
N_FRAMES = N_SAMPLES // HOP_LENGTH           # 3000 mel frames per window
N_AUDIO_CTX = N_FRAMES // 2                  # 1500 encoder positions per window
N_TEXT_CTX = 448                             # decoder context (faster-whisper max_length)


@dataclass(frozen=True)
class SpecialTokens:
    eot: int
    sot: int
    lang_begin: int
    n_langs: int
    translate: int
    transcribe: int
    sot_lm: int
    sot_prev: int
    no_speech: int
    no_timestamps: int
    timestamp_begin: int
    timestamp_end: int
    blank: int = 220                     # " " in the GPT-2 byte-level vocabulary (SuppressBlank)

    def lang_token(self, code: str) -> int:
        idx = LANGUAGES.index(code)
        if idx >= self.n_langs:
            raise ValueError(f"language {code!r} is not in this model's vocabulary")
        return self.lang_begin + idx

    @property
    def lang_codes(self) -> Tuple[str, ...]:
        return LANGUAGES[: self.n_langs]


def special_tokens_for(n_vocab: int, multilingual: bool) -> SpecialTokens:
    """Upstream layout: English-only vocab 51864, multilingual 51865 (99 langs) or 51866 (100 langs)."""
    eot = 50256 if not multilingual else 50257
    n_langs = n_vocab - (eot + 1) - 1 - 6 - N_TIMESTAMPS if multilingual else 0
    if not multilingual:
        # tiny.en layout: eot 50256, sot 50257, translate 50357, transcribe 50358, ...
        n_langs = 99
    sot = eot + 1
    lang_begin = sot + 1
    translate = lang_begin + n_langs
    ts_begin = translate + 6
    st = SpecialTokens(
        eot=eot, sot=sot, lang_begin=lang_begin, n_langs=n_langs if multilingual else 0,
        translate=translate, transcribe=translate + 1, sot_lm=translate + 2, sot_prev=translate + 3,
        no_speech=translate + 4, no_timestamps=translate + 5, timestamp_begin=ts_begin,
        timestamp_end=ts_begin + N_TIMESTAMPS - 1,
    )
    if st.timestamp_end != n_vocab - 1:
        raise ValueError(f"vocab size {n_vocab} does not match the Whisper special-token layout")
    return st


@dataclass(frozen=True)
class ModelDims:
    name: str
    n_mels: int
    n_state: int            # d_model
    n_head: int
    n_enc_layer: int
    n_dec_layer: int
    n_vocab: int
    multilingual: bool
    n_audio_ctx: int = N_AUDIO_CTX
    n_text_ctx: int = N_TEXT_CTX
    # (layer, head) pairs whose cross-attention is used for word alignment
    alignment_heads: Tuple[Tuple[int, int], ...] = field(default=())

    @property
    def n_ffn(self) -> int:
        return 4 * self.n_state

    @property
    def head_dim(self) -> int:
        return self.n_state // self.n_head

    @property
    def specials(self) -> SpecialTokens:
        return special_tokens_for(self.n_vocab, self.multilingual)

    def default_alignment_heads(self) -> Tuple[Tuple[int, int], ...]:
        """Upstream convention when no alignment heads are given: all heads of the last half of the decoder."""
        if self.alignment_heads:
            return self.alignment_heads
        return tuple((l, h) for l in range(self.n_dec_layer // 2, self.n_dec_layer) for h in range(self.n_head))

    # ---- roofline accounting (BASELINE.md "Roofline accounting") ----
    def encoder_flops_per_window(self) -> float:
        d, T, L = self.n_state, self.n_audio_ctx, self.n_enc_layer
        stem = 2 * (2 * T * self.n_mels * 3 * d + T * 3 * d * d)
        return stem + L * 2 * (12 * T * d * d + 2 * T * T * d)

    def cross_kv_flops_per_window(self) -> float:
        return 2 * self.n_dec_layer * 2 * self.n_audio_ctx * self.n_state ** 2

    def decoder_weight_bytes(self) -> float:
        d = self.n_state
        return 2 * (14 * self.n_dec_layer * d * d + self.n_vocab * d)

    def cross_kv_bytes_per_window(self) -> float:
        return self.n_dec_layer * 2 * self.n_audio_ctx * self.n_state * 2

    def self_kv_bytes_per_position(self) -> float:
        return self.n_dec_layer * 2 * self.n_state * 2


_MODELS: Dict[str, ModelDims] = {
    m.name: m
    for m in [
        ModelDims("tiny.en", 80, 384, 6, 4, 4, 51864, False),
        ModelDims("tiny", 80, 384, 6, 4, 4, 51865, True),
        ModelDims("base.en", 80, 512, 8, 6, 6, 51864, False),
        ModelDims("base", 80, 512, 8, 6, 6, 51865, True),
        ModelDims("small.en", 80, 768, 12, 12, 12, 51864, False),
        ModelDims("small", 80, 768, 12, 12, 12, 51865, True),
        ModelDims("medium.en", 80, 1024, 16, 24, 24, 51864, False),
        ModelDims("medium", 80, 1024, 16, 24, 24, 51865, True),
        ModelDims("large-v1", 80, 1280, 20, 32, 32, 51865, True),
        ModelDims("large-v2", 80, 1280, 20, 32, 32, 51865, True),
        ModelDims("large", 80, 1280, 20, 32, 32, 51865, True),
        ModelDims("large-v3", 128, 1280, 20, 32, 32, 51866, True),
        ModelDims("large-v3-turbo", 128, 1280, 20, 32, 4, 51866, True),
    ]
}


def model_dims(name: str) -> ModelDims:
    try:
        return _MODELS[name]
    except KeyError:
        raise ValueError(f"unknown Whisper model {name!r}; known: {sorted(_MODELS)}") from None


def known_models() -> List[str]:
    return sorted(_MODELS)


def custom_dims(name: str, n_mels: int, n_state: int, n_head: int, n_enc_layer: int, n_dec_layer: int,
                n_vocab: int, multilingual: bool, alignment_heads=()) -> ModelDims:
    return ModelDims(name, n_mels, n_state, n_head, n_enc_layer, n_dec_layer, n_vocab, multilingual,
                     alignment_heads=tuple(tuple(x) for x in alignment_heads))
