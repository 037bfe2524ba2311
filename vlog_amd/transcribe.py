"""faster-whisper-shaped drop-in: WhisperModel(...).transcribe(...) -> (Iterable[Segment], TranscriptionInfo).

This is the surface the vlog transcription worker calls (reference `worker/transcription.py:78-111`):

    model = WhisperModel(WHISPER_MODEL, device="cpu", compute_type=TRANSCRIPTION_COMPUTE_TYPE)   # :81-85
    segments, info = model.transcribe(str(wav), language=lang, task="transcribe", beam_size=5,
                                      vad_filter=True)                                          # :105-111
    for segment in segments: segment.start, segment.end, segment.text                           # :117-125
    info.language                                                                               # :131

Semantics follow faster-whisper 1.1.x `WhisperModel.transcribe` / `generate_segments` /
`generate_with_fallback` / `add_word_timestamps` [FW↑] (restated; the package is not installed here):
sequential seek loop over 30 s windows, previous-text prompt (`<|startofprev|>` + last 223 tokens),
temperature fallback on compression ratio / average log-probability with the no-speech exemption, segment
split at timestamp pairs, optional cross-attention word alignment.  Every tensor operation runs on the
MI355X through libwhisper_mi355 (vlog_amd/engine.py); there is no CPU compute path: device="cpu" (the
worker's literal argument) is remapped to the GPU and logged, and construction fails loudly when no GPU or
no HIP library is available.

`BatchedInferencePipeline` is the throughput mode (faster-whisper's class of the same name): fixed 30 s
windows decoded independently (no text conditioning), batched on one GPU, or sharded over several GPUs
with vlog_amd/shard.py.
"""
from __future__ import annotations

import itertools
import logging
import os
import threading
from dataclasses import asdict, dataclass, field
from typing import BinaryIO, Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import segments as segs
from .audio import load_audio
from .dims import CHUNK_LENGTH, HOP_LENGTH, N_FRAMES, SAMPLE_RATE, TIME_PRECISION
from .tokenizer import Tokenizer
from .weights import resolve_model

logger = logging.getLogger("vlog_amd")

FRAMES_PER_SECOND = SAMPLE_RATE // HOP_LENGTH          # 100
INPUT_STRIDE = 2
TOKENS_PER_SECOND = SAMPLE_RATE // (HOP_LENGTH * INPUT_STRIDE)   # 50
MAX_LENGTH = 448


@dataclass
class Word:
    start: float
    end: float
    word: str
    probability: float

    def _asdict(self):
        return asdict(self)


@dataclass
class Segment:
    id: int
    seek: int
    start: float
    end: float
    text: str
    tokens: List[int]
    avg_logprob: float
    compression_ratio: float
    no_speech_prob: float
    words: Optional[List[Word]]
    temperature: Optional[float]

    def _asdict(self):
        return asdict(self)


@dataclass
class TranscriptionOptions:
    beam_size: int
    best_of: int
    patience: float
    length_penalty: float
    repetition_penalty: float
    no_repeat_ngram_size: int
    log_prob_threshold: Optional[float]
    no_speech_threshold: Optional[float]
    compression_ratio_threshold: Optional[float]
    condition_on_previous_text: bool
    prompt_reset_on_temperature: float
    temperatures: List[float]
    initial_prompt: Optional[Union[str, Iterable[int]]]
    prefix: Optional[str]
    suppress_blank: bool
    suppress_tokens: Optional[List[int]]
    without_timestamps: bool
    max_initial_timestamp: float
    word_timestamps: bool
    prepend_punctuations: str
    append_punctuations: str
    multilingual: bool
    max_new_tokens: Optional[int]
    clip_timestamps: Union[str, List[float]]
    hallucination_silence_threshold: Optional[float]
    hotwords: Optional[str]


@dataclass
class VadOptions:
    threshold: float = 0.5
    neg_threshold: Optional[float] = None
    min_speech_duration_ms: int = 0
    max_speech_duration_s: float = float("inf")
    min_silence_duration_ms: int = 2000
    speech_pad_ms: int = 400


@dataclass
class TranscriptionInfo:
    language: str
    language_probability: float
    duration: float
    duration_after_vad: float
    all_language_probs: Optional[List[Tuple[str, float]]]
    transcription_options: TranscriptionOptions
    vad_options: Optional[VadOptions]


@dataclass
class _GenOut:
    tokens: List[int]
    score: float
    no_speech_prob: float


def _resolve_device_index(device: str, device_index) -> int:
    if isinstance(device_index, (list, tuple)):
        if len(device_index) != 1:
            raise ValueError("one WhisperModel drives one GPU; use BatchedInferencePipeline(shards=...) or "
                             "vlog_amd.shard for several")
        device_index = device_index[0]
    env = os.environ.get("VLOG_AMD_DEVICE")
    if env is not None:
        device_index = int(env)
    if device in ("cpu", "auto", "cuda", "rocm", "hip"):
        if device == "cpu":
            logger.warning("WhisperModel(device='cpu') remapped to MI355X GPU %d (vlog_amd has no CPU path)", device_index)
    else:
        raise ValueError(f"unsupported device {device!r}")
    if not torch.cuda.is_available():
        raise RuntimeError("vlog_amd.WhisperModel needs an AMD Instinct GPU (torch.cuda.is_available() is False)")
    return int(device_index)


class WhisperModel:
    """faster_whisper.WhisperModel-compatible constructor (model_size_or_path, device, device_index,
    compute_type, cpu_threads, num_workers, download_root, local_files_only, files, revision, ...)."""

    def __init__(self, model_size_or_path: str, device: str = "auto", device_index: Union[int, List[int]] = 0,
                 compute_type: str = "default", cpu_threads: int = 0, num_workers: int = 1,
                 download_root: Optional[str] = None, local_files_only: bool = False, files: dict = None,
                 revision: Optional[str] = None, use_auth_token=None, seed: int = 0,
                 eot_after: Optional[int] = None, throughput: Optional[bool] = None, vad_model: Optional[str] = None,
                 **model_kwargs):
        """throughput: route transcribe() through BatchedInferencePipeline (default: the VLOG_AMD_THROUGHPUT
        environment variable, so the unchanged worker can opt in without code changes).
        vad_model: Silero VAD v5 weights for vad_filter=True — a local .safetensors/.npz file or
        "synthetic:<seed>" (default: the VLOG_AMD_SILERO_VAD environment variable; unset = the frame-energy
        stand-in, vlog_amd/vad.py)."""
        from .engine import GpuEngine

        if throughput is None:
            throughput = os.environ.get("VLOG_AMD_THROUGHPUT", "0") not in ("", "0")
        self.throughput = bool(throughput)
        self._batched = None

        if files:
            raise NotImplementedError("in-memory model files are not supported")
        if compute_type not in ("default", "auto", "int8", "int8_float16", "int8_float32", "int8_bfloat16",
                                "float16", "bfloat16", "float32"):
            raise ValueError(f"unsupported compute_type {compute_type!r}")
        if compute_type not in ("default", "auto", "bfloat16"):
            logger.info("compute_type=%s mapped to bf16 weights / f32 accumulation on MI355X", compute_type)
        self.device_index = _resolve_device_index(device, device_index)
        self.dims, sd, model_dir = resolve_model(model_size_or_path, seed=seed, eot_after=eot_after)
        self.model_dir = model_dir
        tj = os.path.join(model_dir, "tokenizer.json") if model_dir else None
        self._tokenizer_json = tj if tj and os.path.isfile(tj) else None
        self._tok_seed = seed
        self.engine = GpuEngine(self.dims, sd, self.device_index)
        del sd
        self.engine.reserve(1, 8)
        from .silero import SileroVad, default_spec
        vad_spec = vad_model if vad_model is not None else default_spec()
        self.vad_net = SileroVad.from_spec(self.engine, vad_spec) if vad_spec else None
        self._lock = threading.RLock()
        self.feature_size = self.dims.n_mels
        self.num_samples_per_token = HOP_LENGTH * INPUT_STRIDE
        self.frames_per_second = FRAMES_PER_SECOND
        self.tokens_per_second = TOKENS_PER_SECOND
        self.input_stride = INPUT_STRIDE
        self.time_precision = TIME_PRECISION
        self.max_length = MAX_LENGTH

    def _pipeline(self) -> "BatchedInferencePipeline":
        with self._lock:                      # created once even when several worker threads race here
            if self._batched is None:
                self._batched = BatchedInferencePipeline(
                    self, max_batch_windows=int(os.environ.get("VLOG_AMD_BATCH_WINDOWS", "150")))
            return self._batched

    @property
    def is_multilingual(self) -> bool:
        return self.dims.multilingual

    @property
    def supported_languages(self) -> List[str]:
        return list(self.dims.specials.lang_codes) if self.is_multilingual else ["en"]

    def tokenizer(self, task: Optional[str] = "transcribe", language: Optional[str] = None) -> Tokenizer:
        return Tokenizer(self.dims, task=task, language=language, tokenizer_json=self._tokenizer_json, seed=self._tok_seed)

    # ------------------------------------------------------------------ features / encoder
    def _features(self, audio: np.ndarray) -> torch.Tensor:
        return self.engine.features(torch.from_numpy(np.ascontiguousarray(audio, dtype=np.float32)))

    def _use_cross_form(self, rows_per_window: int) -> None:
        """Cross-attention form for decodes with `rows_per_window` rows per window: the factored form (attention
        over the encoder output; half the bytes of K and V) for one row, the projected K/V form when several
        rows share a window (beam search: every row of the group reads the window's K/V panels once, while the
        factored kernel re-reads the encoder output per 32 (row, head) pairs).  The opt-in fp8
        cross memory is a factored-form mode and is never overridden; VLOG_AMD_CROSS_AUTO=0 disables the choice."""
        if os.environ.get("VLOG_AMD_CROSS_AUTO", "1") == "0" or self.engine.option("cross_fp8", 0):
            return
        self.engine.set_option("cross_mode", 0 if rows_per_window > 1 else 1)

    def _encode(self, features: torch.Tensor, seek: int, size: int, slot: int = 0) -> torch.Tensor:
        enc = self.engine.encode(features, [seek], [size])
        self.engine.cross_kv(enc, slot)
        return enc

    # ------------------------------------------------------------------ language detection
    def detect_language(self, audio: Optional[np.ndarray] = None, features: Optional[torch.Tensor] = None,
                        vad_filter: bool = False, vad_parameters=None, language_detection_segments: int = 1,
                        language_detection_threshold: float = 0.5) -> Tuple[str, float, List[Tuple[str, float]]]:
        """faster-whisper `detect_language`: encode up to `language_detection_segments` windows, one decoder
        step from <|startoftranscript|>, softmax over the language tokens; majority vote if no window is
        confident."""
        if not self.is_multilingual:
            return "en", 1.0, [("en", 1.0)]
        with self._lock:
            if features is None:
                features = self._features(audio)
            st = self.dims.specials
            content = features.shape[1] - 1 if features.shape[1] > 1 else features.shape[1]
            info = {}
            all_probs: List[Tuple[str, float]] = []
            lang, prob = "en", 0.0
            n_seg = max(1, language_detection_segments)
            for i in range(n_seg):
                seek = i * N_FRAMES
                if i > 0 and seek >= content:
                    break
                size = max(0, min(N_FRAMES, content - seek))
                self._encode(features, seek, size, 0)
                p = self.engine.detect_language([0], st.lang_begin, st.n_langs)[0]
                order = np.argsort(-p, kind="stable")
                all_probs = [(st.lang_codes[j], float(p[j])) for j in order]
                lang, prob = all_probs[0]
                if prob > language_detection_threshold:
                    break
                info.setdefault(lang, []).append(prob)
            else:
                lang = max(info, key=lambda k: len(info[k]))
                prob = max(info[lang])
            return lang, prob, all_probs

    # ------------------------------------------------------------------ transcribe
    def transcribe(self, audio: Union[str, BinaryIO, np.ndarray], language: Optional[str] = None,
                   task: str = "transcribe", log_progress: bool = False, beam_size: int = 5, best_of: int = 5,
                   patience: float = 1, length_penalty: float = 1, repetition_penalty: float = 1,
                   no_repeat_ngram_size: int = 0,
                   temperature: Union[float, List[float], Tuple[float, ...]] = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0),
                   compression_ratio_threshold: Optional[float] = 2.4, log_prob_threshold: Optional[float] = -1.0,
                   no_speech_threshold: Optional[float] = 0.6, condition_on_previous_text: bool = True,
                   prompt_reset_on_temperature: float = 0.5, initial_prompt: Optional[Union[str, Iterable[int]]] = None,
                   prefix: Optional[str] = None, suppress_blank: bool = True, suppress_tokens: Optional[List[int]] = [-1],
                   without_timestamps: bool = False, max_initial_timestamp: float = 1.0, word_timestamps: bool = False,
                   prepend_punctuations: str = "\"'“¿([{-", append_punctuations: str = "\"'.。,，!！?？:：”)]}、",
                   multilingual: bool = False, vad_filter: bool = False, vad_parameters=None,
                   max_new_tokens: Optional[int] = None, chunk_length: Optional[int] = None,
                   clip_timestamps: Union[str, List[float]] = "0", hallucination_silence_threshold: Optional[float] = None,
                   hotwords: Optional[str] = None, language_detection_threshold: Optional[float] = 0.5,
                   language_detection_segments: int = 1):
        for name, val, default in (("repetition_penalty", repetition_penalty, 1), ("no_repeat_ngram_size", no_repeat_ngram_size, 0),
                                   ("prefix", prefix, None), ("hotwords", hotwords, None), ("multilingual", multilingual, False),
                                   ("hallucination_silence_threshold", hallucination_silence_threshold, None)):
            if val != default:
                raise NotImplementedError(f"{name}={val!r} is not supported by the MI355X engine")
        if chunk_length not in (None, CHUNK_LENGTH):
            raise NotImplementedError("chunk_length other than 30 s is not supported")
        if task not in ("transcribe", "translate"):
            raise ValueError(f"unknown task {task!r}")
        if self.throughput:
            # opt-in throughput mode for the UNCHANGED worker (VLOG_AMD_THROUGHPUT=1): its call
            # transcribe(wav, language, task, beam_size=5, vad_filter=True) runs as BatchedInferencePipeline:
            # VAD-bounded windows decoded independently in large batches (no previous-text prompt), with
            # timestamps kept so the worker's WebVTT still gets per-segment times.
            if initial_prompt is not None or clip_timestamps not in ("0", [0], [0.0]) or prefix is not None:
                raise NotImplementedError("initial_prompt / clip_timestamps / prefix in throughput mode")
            return self._pipeline().transcribe(
                audio, language=language, task=task, beam_size=beam_size, best_of=best_of, patience=patience,
                length_penalty=length_penalty, temperature=temperature,
                compression_ratio_threshold=compression_ratio_threshold, log_prob_threshold=log_prob_threshold,
                no_speech_threshold=no_speech_threshold, suppress_blank=suppress_blank, suppress_tokens=suppress_tokens,
                without_timestamps=without_timestamps, max_initial_timestamp=max_initial_timestamp,
                word_timestamps=word_timestamps, prepend_punctuations=prepend_punctuations,
                append_punctuations=append_punctuations, vad_filter=vad_filter, vad_parameters=vad_parameters,
                max_new_tokens=max_new_tokens, language_detection_threshold=language_detection_threshold,
                language_detection_segments=language_detection_segments)
        if not isinstance(audio, np.ndarray):
            audio = load_audio(audio)
        audio = np.asarray(audio, dtype=np.float32)
        duration = audio.shape[0] / SAMPLE_RATE
        duration_after_vad = duration
        speech_chunks = None
        vad_opts = None
        if vad_filter and clip_timestamps in ("0", [0], [0.0]):
            from .vad import collect_chunks, get_speech_timestamps
            vad_opts = vad_parameters if isinstance(vad_parameters, VadOptions) else VadOptions(**(vad_parameters or {}))
            speech_chunks = get_speech_timestamps(audio, vad_opts, self)
            audio = collect_chunks(audio, speech_chunks)
            duration_after_vad = audio.shape[0] / SAMPLE_RATE

        with self._lock:
            features = self._features(audio)
        all_language_probs = None
        if language is None:
            if not self.is_multilingual:
                language, language_probability = "en", 1.0
            else:
                language, language_probability, all_language_probs = self.detect_language(
                    features=features, language_detection_segments=language_detection_segments,
                    language_detection_threshold=language_detection_threshold or 0.5)
        else:
            if not self.is_multilingual and language != "en":
                logger.warning("English-only model used with language=%s; using 'en'", language)
                language = "en"
            language_probability = 1.0
        tokenizer = self.tokenizer(task=task, language=language)
        temps = list(temperature) if isinstance(temperature, (list, tuple)) else [temperature]
        options = TranscriptionOptions(
            beam_size=beam_size, best_of=best_of, patience=patience, length_penalty=length_penalty,
            repetition_penalty=repetition_penalty, no_repeat_ngram_size=no_repeat_ngram_size,
            log_prob_threshold=log_prob_threshold, no_speech_threshold=no_speech_threshold,
            compression_ratio_threshold=compression_ratio_threshold, condition_on_previous_text=condition_on_previous_text,
            prompt_reset_on_temperature=prompt_reset_on_temperature, temperatures=temps, initial_prompt=initial_prompt,
            prefix=prefix, suppress_blank=suppress_blank,
            suppress_tokens=list(tokenizer.suppressed_tokens(suppress_tokens)) if suppress_tokens else [],
            without_timestamps=without_timestamps, max_initial_timestamp=max_initial_timestamp,
            word_timestamps=word_timestamps, prepend_punctuations=prepend_punctuations,
            append_punctuations=append_punctuations, multilingual=multilingual, max_new_tokens=max_new_tokens,
            clip_timestamps=clip_timestamps, hallucination_silence_threshold=hallucination_silence_threshold,
            hotwords=hotwords)
        gen = self.generate_segments(features, tokenizer, options)
        if speech_chunks:
            from .vad import restore_speech_timestamps
            gen = restore_speech_timestamps(gen, speech_chunks, SAMPLE_RATE)
        info = TranscriptionInfo(language=language, language_probability=language_probability, duration=duration,
                                 duration_after_vad=duration_after_vad, all_language_probs=all_language_probs,
                                 transcription_options=options, vad_options=vad_opts)
        return gen, info

    # ------------------------------------------------------------------ prompt / generate
    def get_prompt(self, tokenizer: Tokenizer, previous_tokens: List[int], without_timestamps: bool = False) -> List[int]:
        prompt: List[int] = []
        if previous_tokens:
            prompt.append(tokenizer.sot_prev)
            prompt.extend(previous_tokens[-(self.max_length // 2 - 1):])
        prompt.extend(tokenizer.sot_sequence)
        if without_timestamps:
            prompt.append(tokenizer.no_timestamps)
        return prompt

    def _generate(self, prompt: List[int], options: TranscriptionOptions, temperature: float, max_length: int,
                  seed: int) -> _GenOut:
        st = self.dims.specials
        mit = int(round(options.max_initial_timestamp / self.time_precision))
        sampling = temperature > 0
        res, _ = self.engine.generate(
            [0], [prompt], beam_size=1 if sampling else options.beam_size, patience=options.patience,
            length_penalty=options.length_penalty, max_length=max_length, temperature=temperature,
            num_hypotheses=options.best_of if sampling else 1, seed=seed, suppress_tokens=options.suppress_tokens,
            suppress_blank=options.suppress_blank, max_initial_timestamp_index=mit,
            with_timestamps=not options.without_timestamps,
            sot_index=prompt.index(st.sot) if st.sot in prompt else -1, check_every=4)
        r = res[0]
        return _GenOut(r.tokens, r.score, r.no_speech_prob)

    def generate_with_fallback(self, prompt: List[int], tokenizer: Tokenizer, options: TranscriptionOptions,
                               seed: int = 0):
        """faster-whisper generate_with_fallback -> (result, avg_logprob, temperature, compression_ratio)."""
        all_results, below_cr = [], []
        if options.max_new_tokens is not None:
            max_length = len(prompt) + options.max_new_tokens
        else:
            max_length = self.max_length
        if max_length > self.max_length:
            raise ValueError(f"the length of the prompt is {len(prompt)}, and the max_new_tokens {max_length - len(prompt)}. "
                             f"Thus, the combined length of the prompt and max_new_tokens is: {max_length}. This exceeds "
                             f"the max_length of the Whisper model: {self.max_length}.")
        decode_result = None
        temperature = options.temperatures[0] if options.temperatures else 0.0
        for i, temperature in enumerate(options.temperatures):
            result = self._generate(prompt, options, temperature, max_length, seed + i)
            n = len(result.tokens)
            avg_lp = segs.avg_logprob(result.score, n, options.length_penalty)
            text = tokenizer.decode(result.tokens).strip()
            cr = segs.compression_ratio(text)
            decode_result = (result, avg_lp, temperature, cr)
            all_results.append(decode_result)
            fb, below = segs.needs_fallback(cr, avg_lp, result.no_speech_prob, options.compression_ratio_threshold,
                                            options.log_prob_threshold, options.no_speech_threshold)
            if below:
                below_cr.append(decode_result)
            if not fb:
                break
        else:
            best = max(below_cr or all_results, key=lambda x: x[1])
            decode_result = (best[0], best[1], temperature, best[3])
        return decode_result

    # ------------------------------------------------------------------ seek loop
    def generate_segments(self, features: torch.Tensor, tokenizer: Tokenizer, options: TranscriptionOptions):
        content_frames = features.shape[1] - 1
        ct = options.clip_timestamps
        if isinstance(ct, str):
            ct = [float(t) for t in (ct.split(",") if ct else [])]
        seek_points = [round(t * self.frames_per_second) for t in ct]
        if not seek_points:
            seek_points.append(0)
        if len(seek_points) % 2 == 1:
            seek_points.append(content_frames)
        seek_clips = list(zip(seek_points[::2], seek_points[1::2]))
        idx = 0
        clip_idx = 0
        seek = seek_clips[0][0]
        all_tokens: List[int] = []
        prompt_reset_since = 0
        if options.initial_prompt is not None:
            if isinstance(options.initial_prompt, str):
                all_tokens.extend(tokenizer.encode(" " + options.initial_prompt.strip()))
            else:
                all_tokens.extend(options.initial_prompt)
        last_speech_timestamp = 0.0
        window = 0
        while clip_idx < len(seek_clips):
            clip_start, clip_end = seek_clips[clip_idx]
            clip_end = min(clip_end, content_frames)
            if seek < clip_start:
                seek = clip_start
            if seek >= clip_end:
                clip_idx += 1
                if clip_idx < len(seek_clips):
                    seek = seek_clips[clip_idx][0]
                continue
            time_offset = seek * HOP_LENGTH / SAMPLE_RATE
            segment_size = min(N_FRAMES, content_frames - seek, clip_end - seek)
            segment_duration = segment_size * HOP_LENGTH / SAMPLE_RATE
            previous_tokens = all_tokens[prompt_reset_since:]
            # one lock scope from the encode to the word alignment: the alignment reads the window's encoder
            # output from slot 0, which another thread's transcribe must not replace in between
            with self._lock:
                self._use_cross_form(options.beam_size)
                self._encode(features, seek, segment_size, 0)
                prompt = self.get_prompt(tokenizer, previous_tokens, options.without_timestamps)
                result, avg_lp, temperature, cr = self.generate_with_fallback(prompt, tokenizer, options, seed=window)
                skip = segs.should_skip_window(result.no_speech_prob, avg_lp, options.no_speech_threshold,
                                               options.log_prob_threshold)
                if not skip:
                    previous_seek = seek
                    current, seek, single_ending = segs.split_segments_by_timestamps(
                        result.tokens, tokenizer.timestamp_begin, time_offset, segment_size, segment_duration, seek)
                    if options.word_timestamps:
                        last_speech_timestamp = self.add_word_timestamps(
                            [current], tokenizer, segment_size, options.prepend_punctuations,
                            options.append_punctuations, last_speech_timestamp)
            window += 1
            if skip:
                seek += segment_size
                continue
            if options.word_timestamps:
                if not single_ending:
                    last_word_end = _get_end(current)
                    if last_word_end is not None and last_word_end > time_offset:
                        seek = round(last_word_end * self.frames_per_second)
            for s in current:
                text = tokenizer.decode(s["tokens"])
                if s["start"] == s["end"] or not text.strip():
                    continue
                all_tokens.extend(s["tokens"])
                idx += 1
                yield Segment(id=idx, seek=previous_seek, start=s["start"], end=s["end"], text=text,
                              tokens=s["tokens"], temperature=temperature, avg_logprob=avg_lp, compression_ratio=cr,
                              no_speech_prob=result.no_speech_prob,
                              words=[Word(**w) for w in s["words"]] if options.word_timestamps else None)
            if not options.condition_on_previous_text or temperature > options.prompt_reset_on_temperature:
                prompt_reset_since = len(all_tokens)

    # ------------------------------------------------------------------ word timestamps
    def find_alignment(self, tokenizer: Tokenizer, text_tokens: List[List[int]], num_frames: Union[int, Sequence[int]],
                       median_filter_width: int = 7, slots: Optional[Sequence[int]] = None) -> List[List[dict]]:
        """faster-whisper find_alignment over CTranslate2 align: teacher-forced decoder pass over
        [sot_sequence, <|notimestamps|>, text, <|endoftext|>] with the alignment heads' cross-attention
        captured on the GPU, normalise + median filter + DTW on the GPU — every segment group of the call in
        ONE batched align (wm_align_batch).  Group i reads the encoder output in slot slots[i] (default 0) and
        num_frames[i] mel frames (an int applies to every group)."""
        n = len(text_tokens)
        nfs = list(num_frames) if isinstance(num_frames, (list, tuple, np.ndarray)) else [int(num_frames)] * n
        sl = list(slots) if slots is not None else [0] * n
        todo = [i for i in range(n) if text_tokens[i]]
        aligned = dict(zip(todo, self.engine.align_batch([sl[i] for i in todo], tokenizer.sot_sequence,
                                                         [text_tokens[i] for i in todo], [nfs[i] for i in todo],
                                                         self.dims.default_alignment_heads(), median_filter_width)))
        out = []
        for i, tt in enumerate(text_tokens):
            if not tt:
                out.append([])
                continue
            probs, text_idx, time_idx = aligned[i]
            words, word_tokens = tokenizer.split_to_word_tokens(tt + [tokenizer.eot])
            if len(word_tokens) <= 1:
                out.append([])
                continue
            wb = np.pad(np.cumsum([len(t) for t in word_tokens[:-1]]), (1, 0))
            if len(wb) <= 1:
                out.append([])
                continue
            jumps = np.pad(np.diff(text_idx), (1, 0), constant_values=1).astype(bool)
            jump_times = time_idx[jumps] / self.tokens_per_second
            starts = jump_times[wb[:-1]]
            ends = jump_times[wb[1:]]
            wprob = _word_means(probs, wb)
            out.append([dict(word=w, tokens=t, start=float(s), end=float(e), probability=p)
                        for w, t, s, e, p in zip(words, word_tokens, starts, ends, wprob)])
        return out

    def add_word_timestamps(self, segments: List[List[dict]], tokenizer: Tokenizer, num_frames: Union[int, Sequence[int]],
                            prepend_punctuations: str, append_punctuations: str, last_speech_timestamp: float,
                            slots: Optional[Sequence[int]] = None) -> float:
        """faster-whisper add_word_timestamps: segment group i (one window's segments) is aligned against the
        encoder output in slot slots[i] with num_frames[i] frames (BatchedInferencePipeline passes one group
        per window of a batch)."""
        if len(segments) == 0:
            return last_speech_timestamp
        text_tokens, per_seg = [], []
        for segment in segments:
            st = [[t for t in sub["tokens"] if t < tokenizer.eot] for sub in segment]
            text_tokens.append(list(itertools.chain.from_iterable(st)))
            per_seg.append(st)
        alignments = self.find_alignment(tokenizer, text_tokens, num_frames, slots=slots)
        med_max = []
        for alignment in alignments:
            durs = np.array([w["end"] - w["start"] for w in alignment])
            durs = durs[durs.nonzero()]
            med = min(0.7, float(np.median(durs))) if len(durs) > 0 else 0.0
            mx = med * 2
            if len(durs) > 0:
                marks = ".。!！?？"
                for i in range(1, len(alignment)):
                    if alignment[i]["end"] - alignment[i]["start"] > mx:
                        if alignment[i]["word"] in marks:
                            alignment[i]["end"] = alignment[i]["start"] + mx
                        elif alignment[i - 1]["word"] in marks:
                            alignment[i]["start"] = alignment[i]["end"] - mx
            merge_punctuations(alignment, prepend_punctuations, append_punctuations)
            med_max.append((med, mx))
        for si, segment in enumerate(segments):
            wi = 0
            time_offset = segment[0]["seek"] / self.frames_per_second
            med, mx = med_max[si]
            for ssi, sub in enumerate(segment):
                saved = 0
                words = []
                while wi < len(alignments[si]) and saved < len(per_seg[si][ssi]):
                    timing = alignments[si][wi]
                    if timing["word"]:
                        words.append(dict(word=timing["word"], start=round(time_offset + timing["start"], 2),
                                          end=round(time_offset + timing["end"], 2), probability=timing["probability"]))
                    saved += len(timing["tokens"])
                    wi += 1
                if words:
                    if words[0]["end"] - last_speech_timestamp > med * 4 and (
                            words[0]["end"] - words[0]["start"] > mx
                            or (len(words) > 1 and words[1]["end"] - words[0]["start"] > mx * 2)):
                        if len(words) > 1 and words[1]["end"] - words[1]["start"] > mx:
                            boundary = max(words[1]["end"] / 2, words[1]["end"] - mx)
                            words[0]["end"] = words[1]["start"] = boundary
                        words[0]["start"] = max(0, words[0]["end"] - mx)
                    if sub["start"] < words[0]["end"] and sub["start"] - 0.5 > words[0]["start"]:
                        words[0]["start"] = max(0, min(words[0]["end"] - med, sub["start"]))
                    else:
                        sub["start"] = words[0]["start"]
                    if sub["end"] > words[-1]["start"] and sub["end"] + 0.5 < words[-1]["end"]:
                        words[-1]["end"] = max(words[-1]["start"] + med, sub["end"])
                    else:
                        sub["end"] = words[-1]["end"]
                    last_speech_timestamp = sub["end"]
                segments[si][ssi]["words"] = words
        return last_speech_timestamp


def _get_end(segments: List[dict]) -> Optional[float]:
    return next((w["end"] for s in reversed(segments) for w in reversed(s.get("words") or [])),
                segments[-1]["end"] if segments else None)


def _word_means(probs: np.ndarray, wb: np.ndarray) -> List[float]:
    """[float(np.mean(probs[i:j])) ...] over consecutive word boundaries, with np.mean's own arithmetic spelled out for
    float32 (np.add.reduce of the slice, divided by the count in float64, rounded to float32): the same values
    without np.mean's per-call overhead (half the host time of config 5's word probabilities)."""
    p = np.asarray(probs)
    b = np.asarray(wb).tolist()
    if p.dtype != np.float32:
        return [float(np.mean(p[i:j])) for i, j in zip(b[:-1], b[1:])]
    add = np.add.reduce
    return [float(np.float32(float(add(p[i:j])) / (j - i))) if j > i else float(np.mean(p[i:j]))
            for i, j in zip(b[:-1], b[1:])]


def merge_punctuations(alignment: List[dict], prepended: str, appended: str) -> None:
    """faster-whisper / openai merge_punctuations."""
    i = len(alignment) - 2
    j = len(alignment) - 1
    while i >= 0:
        prev, foll = alignment[i], alignment[j]
        if prev["word"].startswith(" ") and prev["word"].strip() in prepended:
            foll["word"] = prev["word"] + foll["word"]
            foll["tokens"] = prev["tokens"] + foll["tokens"]
            prev["word"] = ""
            prev["tokens"] = []
        else:
            j = i
        i -= 1
    i, j = 0, 1
    while j < len(alignment):
        prev, foll = alignment[i], alignment[j]
        if not prev["word"].endswith(" ") and foll["word"] in appended:
            prev["word"] = prev["word"] + foll["word"]
            prev["tokens"] = prev["tokens"] + foll["tokens"]
            foll["word"] = ""
            foll["tokens"] = []
        else:
            i = j
        j += 1


@dataclass
class WindowResult:
    index: int
    seek: int
    size: int
    time_offset: float
    tokens: List[int]
    avg_logprob: float
    temperature: float
    compression_ratio: float
    no_speech_prob: float
    segments: Optional[List[dict]] = None      # split (and, with word timestamps, word-aligned) segments


class BatchedInferencePipeline:
    """Throughput mode (faster-whisper `BatchedInferencePipeline`): the file's 30 s windows — fixed, or bounded
    by VAD speech chunks — are decoded independently (no previous-text prompt) in large batches on one GPU:
    one encoder call per batch, cross-KV for every window resident in HBM, one on-device batched
    greedy/beam decode, then a batched re-decode of the windows that need temperature fallback.
    Window-sharding over several GPUs: vlog_amd/shard.py."""

    def __init__(self, model: WhisperModel, max_batch_windows: int = 150):
        self.model = model
        self.max_batch_windows = max_batch_windows
        # finished windows leave the decode passes (greedy: the row-set decode's compaction; beam: finished windows'
        # hypotheses); VLOG_AMD_COMPACT=0 keeps every row to the batch's end
        self.compact = os.environ.get("VLOG_AMD_COMPACT", "1") != "0"

    # -- windows of the whole-file feature matrix
    @staticmethod
    def fixed_windows(content_frames: int) -> List[Tuple[int, int]]:
        return [(s, min(N_FRAMES, content_frames - s)) for s in range(0, content_frames, N_FRAMES)]

    @staticmethod
    def vad_windows(chunks: List[dict], content_frames: int) -> List[Tuple[int, int]]:
        """Merge speech chunks (sample ranges) greedily into windows of at most 30 s (frame ranges)."""
        out: List[Tuple[int, int]] = []
        cur_s = cur_e = None
        for c in chunks:
            s, e = c["start"] // HOP_LENGTH, min(content_frames, -(-c["end"] // HOP_LENGTH))
            while e - s > N_FRAMES:                          # a single over-long chunk: cut in 30 s pieces
                if cur_s is not None:
                    out.append((cur_s, cur_e - cur_s)); cur_s = None
                out.append((s, N_FRAMES)); s += N_FRAMES
            if cur_s is None:
                cur_s, cur_e = s, e
            elif e - cur_s <= N_FRAMES:
                cur_e = e
            else:
                out.append((cur_s, cur_e - cur_s)); cur_s, cur_e = s, e
        if cur_s is not None and cur_e > cur_s:
            out.append((cur_s, cur_e - cur_s))
        return out

    def decode_windows(self, features: torch.Tensor, windows: Sequence[Tuple[int, int]], time_offsets: Sequence[float],
                       tokenizer: Tokenizer, options: TranscriptionOptions, seed: int = 0,
                       files: Optional[Sequence[int]] = None,
                       seek_bases: Optional[Sequence[int]] = None,
                       last_speech: Optional[dict] = None) -> List[WindowResult]:
        """files: the source file of each window when windows of several files share batches (transcribe_many):
        word timestamps then keep one last-speech time per file.  seek_bases: frame offset of each window's file
        inside `features` (its segments and word timestamps are reported relative to the file).  last_speech:
        the caller's per-file last-speech times (word-timestamp heuristics); owned by ONE transcribe call, so
        threads sharing this pipeline never see each other's state."""
        if last_speech is None:
            last_speech = {}
        m = self.model
        eng = m.engine
        st = m.dims.specials
        prompt = list(tokenizer.sot_sequence) + ([tokenizer.no_timestamps] if options.without_timestamps else [])
        if options.initial_prompt:
            ip = (tokenizer.encode(" " + options.initial_prompt.strip()) if isinstance(options.initial_prompt, str)
                  else list(options.initial_prompt))
            prompt = [tokenizer.sot_prev] + ip[-(m.max_length // 2 - 1):] + prompt
        max_length = min(m.max_length, len(prompt) + options.max_new_tokens) if options.max_new_tokens else m.max_length
        mit = int(round(options.max_initial_timestamp / m.time_precision))
        per = max(options.beam_size, options.best_of, 1)
        # cross-attention form per batch (WhisperModel._use_cross_form), chosen for the FIRST pass: greedy
        # (beam 1) decodes one row per window -> factored; beam groups -> projected (large-v3, 150 windows, beam 5
        # + words: 1474 vs 1237 RTFx).  The temperature-fallback passes (best_of rows) reuse the batch's form.
        auto_form = os.environ.get("VLOG_AMD_CROSS_AUTO", "1") != "0" and not eng.option("cross_fp8", 0)
        prev_form = eng.option("cross_mode")
        try:
            return self._decode_batches(features, windows, time_offsets, tokenizer, options, seed, files, seek_bases,
                                        last_speech, prompt, max_length, mit, per, auto_form)
        finally:
            if auto_form:                      # leave the engine in the form the caller had configured
                with m._lock:
                    eng.set_option("cross_mode", 1 if prev_form is None else prev_form)

    def _decode_batches(self, features, windows, time_offsets, tokenizer, options, seed, files, seek_bases,
                        last_speech, prompt, max_length, mit, per, auto_form) -> List[WindowResult]:
        m = self.model
        eng = m.engine
        st = m.dims.specials
        out: List[WindowResult] = []
        B = self.max_batch_windows
        for b0 in range(0, len(windows), B):
            wins = list(windows[b0: b0 + B])
            with m._lock:
                if auto_form:
                    m._use_cross_form(options.beam_size)
                eng.reserve(len(wins), len(wins) * per)
                enc = eng.encode(features, [w[0] for w in wins], [w[1] for w in wins])
                eng.cross_kv(enc, 0)
                del enc
                pending = list(range(len(wins)))
                results: dict = {}
                tries: dict = {i: [] for i in pending}
                for ti, T in enumerate(options.temperatures):
                    if not pending:
                        break
                    sampling = T > 0
                    res, _ = eng.generate(
                        pending, [prompt] * len(pending), beam_size=1 if sampling else options.beam_size,
                        patience=options.patience, length_penalty=options.length_penalty, max_length=max_length,
                        temperature=T, num_hypotheses=options.best_of if sampling else 1, seed=seed + 7919 * ti + b0,
                        suppress_tokens=options.suppress_tokens, suppress_blank=options.suppress_blank,
                        max_initial_timestamp_index=mit, with_timestamps=not options.without_timestamps,
                        sot_index=prompt.index(st.sot), check_every=4, compact=self.compact)
                    still = []
                    for i, r in zip(pending, res):
                        alp = segs.avg_logprob(r.score, len(r.tokens), options.length_penalty)
                        cr = segs.compression_ratio(tokenizer.decode(r.tokens).strip())
                        fb, below = segs.needs_fallback(cr, alp, r.no_speech_prob, options.compression_ratio_threshold,
                                                        options.log_prob_threshold, options.no_speech_threshold)
                        tries[i].append((r, alp, T, cr, below))
                        if fb:
                            still.append(i)
                        else:
                            results[i] = (r, alp, T, cr)
                    pending = still
                for i in pending:                      # every temperature failed: best avg logprob
                    cand = [t for t in tries[i] if t[4]] or tries[i]
                    r, alp, _, cr, _ = max(cand, key=lambda t: t[1])
                    results[i] = (r, alp, options.temperatures[-1], cr)
                batch = []
                for i, (s, n) in enumerate(wins):
                    r, alp, T, cr = results[i]
                    sb = seek_bases[b0 + i] if seek_bases is not None else 0
                    wr = WindowResult(b0 + i, s - sb, n, time_offsets[b0 + i], r.tokens, alp, T, cr, r.no_speech_prob)
                    wr.segments = self.window_segments(wr, tokenizer, options)
                    batch.append(wr)
                if options.word_timestamps:
                    # the batch's encoder outputs are still in slots 0..B-1: one batched alignment for every
                    # window with text (faster-whisper aligns a whole batch of segments in one model.align); with
                    # several files, one call per file so each keeps its own last-speech time
                    fid = [files[b0 + i] if files is not None else 0 for i in range(len(batch))]
                    for f in sorted(set(fid)):
                        idx = [i for i, wr in enumerate(batch) if wr.segments and fid[i] == f]
                        if idx:
                            last_speech[f] = m.add_word_timestamps(
                                [batch[i].segments for i in idx], tokenizer, [batch[i].size for i in idx],
                                options.prepend_punctuations, options.append_punctuations,
                                last_speech.get(f, 0.0), slots=idx)
                out.extend(batch)
        return out

    def window_segments(self, wr: WindowResult, tokenizer: Tokenizer, options: TranscriptionOptions) -> List[dict]:
        if segs.should_skip_window(wr.no_speech_prob, wr.avg_logprob, options.no_speech_threshold,
                                   options.log_prob_threshold):
            return []
        dur = wr.size * HOP_LENGTH / SAMPLE_RATE
        if options.without_timestamps:
            cur = [dict(seek=wr.seek, start=wr.time_offset, end=wr.time_offset + dur,
                        tokens=[t for t in wr.tokens if t < tokenizer.eot])]
        else:
            cur, _, _ = segs.split_segments_by_timestamps(wr.tokens, tokenizer.timestamp_begin, wr.time_offset,
                                                          wr.size, dur, wr.seek)
        return cur

    def transcribe(self, audio: Union[str, BinaryIO, np.ndarray], language: Optional[str] = None,
                   task: str = "transcribe", log_progress: bool = False, beam_size: int = 5, best_of: int = 5,
                   patience: float = 1, length_penalty: float = 1, repetition_penalty: float = 1,
                   no_repeat_ngram_size: int = 0,
                   temperature: Union[float, List[float], Tuple[float, ...]] = (0.0, 0.2, 0.4, 0.6, 0.8, 1.0),
                   compression_ratio_threshold: Optional[float] = 2.4, log_prob_threshold: Optional[float] = -1.0,
                   no_speech_threshold: Optional[float] = 0.6, initial_prompt=None, prefix: Optional[str] = None,
                   suppress_blank: bool = True, suppress_tokens: Optional[List[int]] = [-1],
                   without_timestamps: bool = True, max_initial_timestamp: float = 1.0, word_timestamps: bool = False,
                   prepend_punctuations: str = "\"'“¿([{-", append_punctuations: str = "\"'.。,，!！?？:：”)]}、",
                   multilingual: bool = False, vad_filter: bool = True, vad_parameters=None,
                   max_new_tokens: Optional[int] = None, chunk_length: Optional[int] = None, clip_timestamps=None,
                   hallucination_silence_threshold: Optional[float] = None, batch_size: int = 16,
                   hotwords: Optional[str] = None, language_detection_threshold: Optional[float] = 0.5,
                   language_detection_segments: int = 1):
        for name, val, default in (("repetition_penalty", repetition_penalty, 1), ("no_repeat_ngram_size", no_repeat_ngram_size, 0),
                                   ("prefix", prefix, None), ("hotwords", hotwords, None), ("multilingual", multilingual, False),
                                   ("hallucination_silence_threshold", hallucination_silence_threshold, None)):
            if val != default:
                raise NotImplementedError(f"{name}={val!r} is not supported by the MI355X engine")
        prep = self._prepare(audio, language, vad_filter, vad_parameters, language_detection_segments,
                             language_detection_threshold)
        tokenizer = self.model.tokenizer(task=task, language=prep["language"])
        options = self._options(
            tokenizer, beam_size=beam_size, best_of=best_of, patience=patience, length_penalty=length_penalty,
            temperature=temperature, compression_ratio_threshold=compression_ratio_threshold,
            log_prob_threshold=log_prob_threshold, no_speech_threshold=no_speech_threshold,
            initial_prompt=initial_prompt, suppress_blank=suppress_blank, suppress_tokens=suppress_tokens,
            without_timestamps=without_timestamps, max_initial_timestamp=max_initial_timestamp,
            word_timestamps=word_timestamps, prepend_punctuations=prepend_punctuations,
            append_punctuations=append_punctuations, max_new_tokens=max_new_tokens, clip_timestamps=clip_timestamps)
        windows = prep["windows"]
        offsets = [s * HOP_LENGTH / SAMPLE_RATE for s, _ in windows]
        results = self.decode_windows(prep["features"], windows, offsets, tokenizer, options, last_speech={})
        return self._segments(prep["features"], results, tokenizer, options), self._info(prep, options)

    def transcribe_many(self, audios: Sequence[Union[str, BinaryIO, np.ndarray]],
                        language: Union[None, str, Sequence[Optional[str]]] = None, task: str = "transcribe",
                        vad_filter: bool = True, vad_parameters=None, language_detection_segments: int = 1,
                        language_detection_threshold: Optional[float] = 0.5, **kw):
        """Several files in shared decode batches: the worker transcribes one video at a time
        (reference worker/transcription.py:496-506), so a short file leaves most of a 150-window batch empty.
        Here the windows of all files (same task; grouped by language, since the prompt carries it) are packed
        into the same batches: the files' log-mel matrices are concatenated along time (each normalised with
        its own global max, as faster-whisper does per file) and every window keeps its file's time offsets.
        Returns [(segments, info)] per file, in input order; each file's result is what `transcribe` gives for
        it alone (same windows, prompts and options)."""
        n = len(audios)
        langs = list(language) if isinstance(language, (list, tuple)) else [language] * n
        if len(langs) != n:
            raise ValueError("one language per file")
        preps = [self._prepare(a, l, vad_filter, vad_parameters, language_detection_segments,
                               language_detection_threshold) for a, l in zip(audios, langs)]
        out: List[Optional[tuple]] = [None] * n
        last_speech: dict = {}
        for lang in sorted({p["language"] for p in preps}):
            files = [i for i, p in enumerate(preps) if p["language"] == lang]
            tokenizer = self.model.tokenizer(task=task, language=lang)
            options = self._options(tokenizer, **kw)
            feats = torch.cat([preps[i]["features"] for i in files], dim=1) if len(files) > 1 else preps[files[0]]["features"]
            windows, offsets, fids, bases = [], [], [], {}
            base = 0
            for i in files:
                bases[i] = base
                for s, nf in preps[i]["windows"]:
                    windows.append((base + s, nf))
                    offsets.append(s * HOP_LENGTH / SAMPLE_RATE)
                    fids.append(i)
                base += preps[i]["features"].shape[1]
            results = self.decode_windows(feats, windows, offsets, tokenizer, options, files=fids,
                                          seek_bases=[bases[f] for f in fids], last_speech=last_speech)
            for i in files:
                mine = [wr for wr, f in zip(results, fids) if f == i]
                out[i] = (list(self._segments(None, mine, tokenizer, options)), self._info(preps[i], options))
        return out

    def _prepare(self, audio, language, vad_filter, vad_parameters, language_detection_segments,
                 language_detection_threshold) -> dict:
        """One file: PCM, log-mel, its windows (VAD-bounded or fixed) and its language.  `audio` may be an
        IngestResult (vlog_amd/ingest.py: PCM and log-mel already on the device, computed while streaming)."""
        from .ingest import IngestResult
        m = self.model
        if isinstance(audio, IngestResult):
            features, duration = audio.features, audio.duration
            audio = audio.pcm
        else:
            if not isinstance(audio, np.ndarray):
                audio = load_audio(audio)
            audio = np.asarray(audio, dtype=np.float32)
            duration = audio.shape[0] / SAMPLE_RATE
            with m._lock:
                features = m._features(audio)
        content = features.shape[1] - 1
        vad_opts = None
        if vad_filter:
            from .vad import get_speech_timestamps
            vad_opts = vad_parameters if isinstance(vad_parameters, VadOptions) else VadOptions(**(vad_parameters or {}))
            chunks = get_speech_timestamps(audio, vad_opts, m)
            windows = self.vad_windows(chunks, content)
            duration_after_vad = sum(c["end"] - c["start"] for c in chunks) / SAMPLE_RATE
        else:
            windows = self.fixed_windows(content)
            duration_after_vad = duration
        all_language_probs = None
        if language is None:
            if m.is_multilingual and windows:
                language, language_probability, all_language_probs = m.detect_language(
                    features=features, language_detection_segments=language_detection_segments,
                    language_detection_threshold=language_detection_threshold or 0.5)
            else:
                language, language_probability = "en", 1.0
        else:
            language_probability = 1.0
        return dict(features=features, windows=windows, duration=duration, duration_after_vad=duration_after_vad,
                    vad_opts=vad_opts, language=language, language_probability=language_probability,
                    all_language_probs=all_language_probs)

    @staticmethod
    def _options(tokenizer: Tokenizer, beam_size: int = 5, best_of: int = 5, patience: float = 1,
                 length_penalty: float = 1, temperature=(0.0, 0.2, 0.4, 0.6, 0.8, 1.0),
                 compression_ratio_threshold: Optional[float] = 2.4, log_prob_threshold: Optional[float] = -1.0,
                 no_speech_threshold: Optional[float] = 0.6, initial_prompt=None, suppress_blank: bool = True,
                 suppress_tokens: Optional[List[int]] = [-1], without_timestamps: bool = True,
                 max_initial_timestamp: float = 1.0, word_timestamps: bool = False,
                 prepend_punctuations: str = "\"'“¿([{-", append_punctuations: str = "\"'.。,，!！?？:：”)]}、",
                 max_new_tokens: Optional[int] = None, clip_timestamps=None) -> TranscriptionOptions:
        temps = list(temperature) if isinstance(temperature, (list, tuple)) else [temperature]
        return TranscriptionOptions(
            beam_size=beam_size, best_of=best_of, patience=patience, length_penalty=length_penalty,
            repetition_penalty=1, no_repeat_ngram_size=0,
            log_prob_threshold=log_prob_threshold, no_speech_threshold=no_speech_threshold,
            compression_ratio_threshold=compression_ratio_threshold, condition_on_previous_text=False,
            prompt_reset_on_temperature=0.5, temperatures=temps, initial_prompt=initial_prompt, prefix=None,
            suppress_blank=suppress_blank,
            suppress_tokens=list(tokenizer.suppressed_tokens(suppress_tokens)) if suppress_tokens else [],
            without_timestamps=without_timestamps, max_initial_timestamp=max_initial_timestamp,
            word_timestamps=word_timestamps, prepend_punctuations=prepend_punctuations,
            append_punctuations=append_punctuations, multilingual=False, max_new_tokens=max_new_tokens,
            clip_timestamps=clip_timestamps or "0", hallucination_silence_threshold=None, hotwords=None)

    @staticmethod
    def _info(prep: dict, options: TranscriptionOptions) -> TranscriptionInfo:
        return TranscriptionInfo(language=prep["language"], language_probability=prep["language_probability"],
                                 duration=prep["duration"], duration_after_vad=prep["duration_after_vad"],
                                 all_language_probs=prep["all_language_probs"], transcription_options=options,
                                 vad_options=prep["vad_opts"])

    def _segments(self, features, results: List[WindowResult], tokenizer: Tokenizer, options: TranscriptionOptions):
        idx = 0
        for wr in results:
            cur = wr.segments if wr.segments is not None else self.window_segments(wr, tokenizer, options)
            for s in cur:
                text = tokenizer.decode(s["tokens"])
                if s["start"] == s["end"] or not text.strip():
                    continue
                idx += 1
                yield Segment(id=idx, seek=wr.seek, start=s["start"], end=s["end"], text=text, tokens=s["tokens"],
                              avg_logprob=wr.avg_logprob, compression_ratio=wr.compression_ratio,
                              no_speech_prob=wr.no_speech_prob, temperature=wr.temperature,
                              words=[Word(**w) for w in s["words"]] if options.word_timestamps else None)


def default_batched_options(**kw) -> dict:
    """TranscriptionOptions fields (as a dict) for the batched/sharded throughput mode."""
    base = dict(beam_size=5, best_of=5, patience=1.0, length_penalty=1.0, repetition_penalty=1.0,
                no_repeat_ngram_size=0, log_prob_threshold=-1.0, no_speech_threshold=0.6,
                compression_ratio_threshold=2.4, condition_on_previous_text=False, prompt_reset_on_temperature=0.5,
                temperatures=[0.0, 0.2, 0.4, 0.6, 0.8, 1.0], initial_prompt=None, prefix=None, suppress_blank=True,
                suppress_tokens=[-1], without_timestamps=False, max_initial_timestamp=1.0, word_timestamps=False,
                prepend_punctuations="\"'“¿([{-", append_punctuations="\"'.。,，!！?？:：”)]}、", multilingual=False,
                max_new_tokens=None, clip_timestamps="0", hallucination_silence_threshold=None, hotwords=None)
    if "temperature" in kw:
        t = kw.pop("temperature")
        kw["temperatures"] = list(t) if isinstance(t, (list, tuple)) else [t]
    unknown = set(kw) - set(base)
    if unknown:
        raise TypeError(f"unknown options {sorted(unknown)}")
    base.update(kw)
    return base
