"""GPU engine wrapper: packs weights into the C-ABI layout and calls libwhisper_mi355 on one MI355X.

PyTorch-ROCm is plumbing here: it allocates the device buffers the C-ABI reads and writes and provides the
stream.  All arithmetic runs in the hand-written gfx950 kernels behind vlog_amd/_capi.py.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _capi
from .dims import ModelDims, N_FRAMES, HOP_LENGTH


def _i32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _f32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


@dataclass
class GenResult:
    tokens: List[int]
    score: float
    cum_logprob: float
    no_speech_prob: float
    # per-step records (generate(record_logprobs=True)): log-prob of the token chosen at each step, the final
    # <|endoftext|> included when the window ended on it; greedy / sampling also the best other allowed token's
    token_logprobs: Optional[np.ndarray] = None
    token_logprobs_other: Optional[np.ndarray] = None


def pack_weights(dims: ModelDims, sd: Dict[str, torch.Tensor], device) -> Dict[str, torch.Tensor]:
    """HF-named float32 weights -> the engine's packed names/layouts (include/whisper_mi355.h)."""
    d, m = dims.n_state, dims.n_mels
    k1p = ((3 * m + 63) // 64) * 64
    bf, f32 = torch.bfloat16, torch.float32
    out: Dict[str, torch.Tensor] = {}

    def g(n):
        return sd[n].to(device=device, dtype=f32)

    w1 = g("model.encoder.conv1.weight").permute(0, 2, 1).reshape(d, 3 * m)
    out["enc.conv1.w"] = torch.nn.functional.pad(w1, (0, k1p - 3 * m)).to(bf).contiguous()
    out["enc.conv1.b"] = g("model.encoder.conv1.bias")
    out["enc.conv2.w"] = g("model.encoder.conv2.weight").permute(0, 2, 1).reshape(d, 3 * d).to(bf).contiguous()
    out["enc.conv2.b"] = g("model.encoder.conv2.bias")
    out["enc.pos"] = g("model.encoder.embed_positions.weight")[: dims.n_audio_ctx].contiguous()
    zeros = torch.zeros(d, device=device, dtype=f32)

    def attn(dst, src):
        out[dst + "qkv.w"] = torch.cat([g(src + "q_proj.weight"), g(src + "k_proj.weight"), g(src + "v_proj.weight")]).to(bf).contiguous()
        out[dst + "qkv.b"] = torch.cat([g(src + "q_proj.bias"), zeros, g(src + "v_proj.bias")]).contiguous()
        out[dst + "out.w"] = g(src + "out_proj.weight").to(bf).contiguous()
        out[dst + "out.b"] = g(src + "out_proj.bias")

    def ln(dst, src):
        out[dst + ".w"] = g(src + ".weight")
        out[dst + ".b"] = g(src + ".bias")

    def mlp(dst, src):
        out[dst + "fc1.w"] = g(src + "fc1.weight").to(bf).contiguous()
        out[dst + "fc1.b"] = g(src + "fc1.bias")
        out[dst + "fc2.w"] = g(src + "fc2.weight").to(bf).contiguous()
        out[dst + "fc2.b"] = g(src + "fc2.bias")

    for l in range(dims.n_enc_layer):
        s, t = f"model.encoder.layers.{l}.", f"enc.{l}."
        attn(t, s + "self_attn.")
        ln(t + "ln1", s + "self_attn_layer_norm")
        ln(t + "ln2", s + "final_layer_norm")
        mlp(t, s)
    ln("enc.ln", "model.encoder.layer_norm")
    out["dec.embed"] = g("model.decoder.embed_tokens.weight").to(bf).contiguous()
    out["dec.pos"] = g("model.decoder.embed_positions.weight")[: dims.n_text_ctx].contiguous()
    ckv_w, ckv_b = [], []
    for l in range(dims.n_dec_layer):
        s, t = f"model.decoder.layers.{l}.", f"dec.{l}."
        attn(t, s + "self_attn.")
        ln(t + "ln1", s + "self_attn_layer_norm")
        ln(t + "ln2", s + "encoder_attn_layer_norm")
        ln(t + "ln3", s + "final_layer_norm")
        out[t + "cq.w"] = g(s + "encoder_attn.q_proj.weight").to(bf).contiguous()
        out[t + "cq.b"] = g(s + "encoder_attn.q_proj.bias")
        out[t + "cout.w"] = g(s + "encoder_attn.out_proj.weight").to(bf).contiguous()
        out[t + "cout.b"] = g(s + "encoder_attn.out_proj.bias")
        mlp(t, s)
        ckv_w += [g(s + "encoder_attn.k_proj.weight"), g(s + "encoder_attn.v_proj.weight")]
        ckv_b += [zeros, g(s + "encoder_attn.v_proj.bias")]
    out["dec.ckv.w"] = torch.cat(ckv_w).to(bf).contiguous()
    out["dec.ckv.b"] = torch.cat(ckv_b).contiguous()
    ln("dec.ln", "model.decoder.layer_norm")
    return out


class GpuEngine:
    """One engine per GPU process.  Thread-safe (the C-ABI serialises calls and sets the device itself)."""

    def __init__(self, dims: ModelDims, state_dict: Dict[str, torch.Tensor], device_index: int = 0):
        self.lib = _capi.load()
        self.dims = dims
        self.device = torch.device("cuda", device_index)
        st = dims.specials
        cd = _capi.ModelDimsC(dims.n_mels, dims.n_state, dims.n_head, dims.n_enc_layer, dims.n_dec_layer,
                              dims.n_vocab, dims.n_audio_ctx, dims.n_text_ctx, st.eot, st.sot, st.no_speech,
                              st.no_timestamps, st.timestamp_begin, st.blank)
        h = C.c_void_p()
        _capi.check(self.lib.wm_create(C.byref(cd), device_index, C.byref(h)), "wm_create")
        self.h = h
        self.n_slots = 0
        self.n_hyp = 0
        with torch.cuda.device(self.device):
            packed = pack_weights(dims, state_dict, self.device)
            s = self.stream_ptr()
            for name, t in packed.items():
                _capi.check(self.lib.wm_set_weight(self.h, name.encode(), C.c_void_p(t.data_ptr()),
                                                   t.numel() * t.element_size(), s), f"wm_set_weight({name})")
            torch.cuda.synchronize(self.device)
            del packed
        if not self.lib.wm_weights_complete(self.h):
            raise RuntimeError("engine weights incomplete")

    @classmethod
    def frontend(cls, dims: ModelDims, device_index: int = 0) -> "GpuEngine":
        """An engine handle with NO weights loaded, for the front end alone (log-mel, frame energy, VAD): a shard
        coordinator needs the features (and the global log-mel max) before any model pass.  wm_create builds the
        n_mels filterbank, so features() runs the same kernels as a full engine of these dims; the decoder and
        encoder entry points fail (wm_weights_complete is false)."""
        self = cls.__new__(cls)
        self.lib = _capi.load()
        self.dims = dims
        self.device = torch.device("cuda", device_index)
        st = dims.specials
        cd = _capi.ModelDimsC(dims.n_mels, dims.n_state, dims.n_head, dims.n_enc_layer, dims.n_dec_layer,
                              dims.n_vocab, dims.n_audio_ctx, dims.n_text_ctx, st.eot, st.sot, st.no_speech,
                              st.no_timestamps, st.timestamp_begin, st.blank)
        h = C.c_void_p()
        _capi.check(self.lib.wm_create(C.byref(cd), device_index, C.byref(h)), "wm_create")
        self.h = h
        self.n_slots = 0
        self.n_hyp = 0
        return self

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.wm_destroy(h)
            except Exception:
                pass
            self.h = None

    def stream_ptr(self) -> C.c_void_p:
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def profile(self, enable: bool, classes: Optional[Sequence[str]] = None) -> None:
        """Reset + enable the built-in event profiler (all classes, or only `classes`); False disables."""
        if not enable:
            _capi.check(self.lib.wm_profile_select(self.h, 0), "wm_profile_select")
            return
        if classes is None:
            _capi.check(self.lib.wm_profile(self.h, 1), "wm_profile")
            return
        names = [self.lib.wm_profile_name(c).decode() for c in range(self.lib.wm_profile_classes())]
        mask = 0
        for n in classes:
            mask |= 1 << names.index(n)
        _capi.check(self.lib.wm_profile_select(self.h, mask), "wm_profile_select")

    def profile_read(self) -> Dict[str, dict]:
        out = {}
        for c in range(self.lib.wm_profile_classes()):
            n, ms, fl, by = C.c_int64(), C.c_double(), C.c_double(), C.c_double()
            _capi.check(self.lib.wm_profile_read(self.h, c, C.byref(n), C.byref(ms), C.byref(fl), C.byref(by)), "wm_profile_read")
            out[self.lib.wm_profile_name(c).decode()] = dict(launches=n.value, ms=ms.value, flops=fl.value, bytes=by.value)
        return out

    def encoder_attention(self, qkv: torch.Tensor) -> torch.Tensor:
        """The encoder self-attention kernel alone: qkv bf16 [B, T, 3d] -> bf16 [B, T, d] (diagnostics/tests)."""
        B, T, three_d = qkv.shape
        if qkv.dtype != torch.bfloat16 or three_d != 3 * self.dims.n_state or not qkv.is_contiguous():
            raise ValueError("encoder_attention: qkv must be contiguous bf16 [B, T, 3 n_state]")
        out = torch.empty(B, T, self.dims.n_state, dtype=torch.bfloat16, device=self.device)
        _capi.check(self.lib.wm_encoder_attention(self.h, C.c_void_p(qkv.data_ptr()), C.c_void_p(out.data_ptr()),
                                                  B, T, self.stream_ptr()), "wm_encoder_attention")
        return out

    def cross_fp8_quantize(self, enc: torch.Tensor):
        """wm_cross_fp8_quantize on bf16 rows [..., n_state] -> (uint8 codes, f32 scale per row), device tensors."""
        x = enc.reshape(-1, enc.shape[-1]).contiguous()
        codes = torch.empty(x.shape, dtype=torch.uint8, device=self.device)
        scale = torch.empty(x.shape[0], dtype=torch.float32, device=self.device)
        _capi.check(self.lib.wm_cross_fp8_quantize(self.h, C.c_void_p(x.data_ptr()), x.shape[0],
                                                    C.c_void_p(codes.data_ptr()), C.c_void_p(scale.data_ptr()),
                                                    self.stream_ptr()), "wm_cross_fp8_quantize")
        return codes, scale

    def set_option(self, key: str, value: int) -> None:
        """Engine scheduling knob (wm_set_option), e.g. set_option("decode_split", 0)."""
        _capi.check(self.lib.wm_set_option(self.h, key.encode(), int(value)), "wm_set_option")

    def option(self, key: str, default: Optional[int] = None) -> Optional[int]:
        """The engine's current value of an option (wm_get_option: includes environment overrides and defaults);
        `default` only for keys the engine does not know."""
        v = C.c_int64()
        if self.lib.wm_get_option(self.h, key.encode(), C.byref(v)) != 0:
            if default is not None:
                return default
            _capi.check(-1, f"wm_get_option({key})")
        return int(v.value)

    def device_bytes(self) -> int:
        return int(self.lib.wm_device_bytes(self.h))

    # ------------------------------------------------------------------ log-mel
    def logmel(self, pcm: torch.Tensor, n_samples: Optional[int] = None, pcm_offset: int = 0, frame0: int = 0,
               n_frames: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Unclamped log10 mel of frames [frame0, frame0+n_frames) of a file of n_samples samples.
        -> (mel f32 [n_mels, n_frames] on device, gmax uint32 [1] ordered-max accumulator)."""
        if n_samples is None:
            n_samples = pcm.numel()
        if n_frames is None:
            n_frames = (n_samples + HOP_LENGTH) // HOP_LENGTH - frame0
        pcm = pcm.to(self.device, torch.float32).contiguous()
        mel = torch.empty((self.dims.n_mels, max(n_frames, 1)), device=self.device, dtype=torch.float32)
        gmax = torch.zeros(1, device=self.device, dtype=torch.int32)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_logmel(self.h, C.c_void_p(pcm.data_ptr()), pcm_offset, n_samples, frame0, n_frames,
                                           C.c_void_p(mel.data_ptr()), mel.shape[1], C.c_void_p(gmax.data_ptr()),
                                           self.stream_ptr()), "wm_logmel")
        return mel, gmax

    def logmel_finalize(self, mel: torch.Tensor, gmax: torch.Tensor, gmax_value: Optional[float] = None) -> float:
        hv = (C.c_float * 1)(gmax_value) if gmax_value is not None else None
        out = (C.c_float * 1)()
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_logmel_finalize(self.h, C.c_void_p(mel.data_ptr()), mel.shape[1], mel.shape[1],
                                                    C.c_void_p(gmax.data_ptr()),
                                                    C.cast(hv, C.POINTER(C.c_float)) if hv is not None else None,
                                                    C.cast(out, C.POINTER(C.c_float)), self.stream_ptr()),
                        "wm_logmel_finalize")
        return float(out[0])

    def gmax_value(self, gmax: torch.Tensor) -> float:
        u = int(gmax.cpu().view(torch.int32).numpy().astype(np.uint32)[0])
        u = (u & 0x7FFFFFFF) if (u & 0x80000000) else (~u & 0xFFFFFFFF)
        return float(np.array([u], dtype=np.uint32).view(np.float32)[0])

    def frame_energy_db(self, pcm: torch.Tensor, frame: int = 512) -> np.ndarray:
        pcm = pcm.to(self.device, torch.float32).contiguous()
        n = pcm.numel()
        out = torch.empty(max(1, (n + frame - 1) // frame), device=self.device, dtype=torch.float32)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_frame_energy(self.h, C.c_void_p(pcm.data_ptr()), n, frame, C.c_void_p(out.data_ptr()),
                                                 self.stream_ptr()), "wm_frame_energy")
        return out.cpu().numpy()[: (n + frame - 1) // frame]

    def features(self, pcm: torch.Tensor) -> torch.Tensor:
        """faster-whisper FeatureExtractor(audio): clamped log-mel [n_mels, N//160 + 1] on device."""
        mel, gmax = self.logmel(pcm)
        self.logmel_finalize(mel, gmax)
        return mel

    # ------------------------------------------------------------------ encoder / decoder
    def encode(self, mel: torch.Tensor, seeks: Sequence[int], nframes: Sequence[int]) -> torch.Tensor:
        B = len(seeks)
        s = np.ascontiguousarray(seeks, dtype=np.int32)
        n = np.ascontiguousarray(nframes, dtype=np.int32)
        enc = torch.empty((B, self.dims.n_audio_ctx, self.dims.n_state), device=self.device, dtype=torch.bfloat16)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_encode(self.h, C.c_void_p(mel.data_ptr()), mel.shape[1], _i32p(s), _i32p(n), B,
                                           C.c_void_p(enc.data_ptr()), self.stream_ptr()), "wm_encode")
        return enc

    def reserve(self, n_slots: int, n_hyp: int) -> None:
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_reserve(self.h, n_slots, n_hyp, self.stream_ptr()), "wm_reserve")
        self.n_slots = max(self.n_slots, n_slots)
        self.n_hyp = max(self.n_hyp, n_hyp)

    def cross_kv(self, enc: torch.Tensor, slot0: int = 0) -> None:
        B = enc.shape[0]
        if slot0 + B > self.n_slots:
            self.reserve(slot0 + B, max(self.n_hyp, 1))
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_cross_kv(self.h, C.c_void_p(enc.data_ptr()), B, slot0, self.stream_ptr()), "wm_cross_kv")

    def generate(self, slots: Sequence[int], prompts: Sequence[Sequence[int]], *, beam_size: int = 1,
                 patience: float = 1.0, length_penalty: float = 1.0, max_length: int = 448,
                 temperature: float = 0.0, num_hypotheses: int = 1, seed: int = 0,
                 suppress_tokens: Sequence[int] = (), suppress_blank: bool = True,
                 max_initial_timestamp_index: Optional[int] = 50, with_timestamps: bool = True,
                 sot_index: Optional[int] = None, check_every: int = 4, max_rows: int = 0, compact: bool = False,
                 record_logprobs: bool = False, stats: Optional[dict] = None) -> Tuple[List[GenResult], int]:
        """ctranslate2 Whisper.generate over windows in slots (wm_generate).  max_rows / compact: the row-set decode
        (greedy / one sampled hypothesis; windows refill finished rows in the given order, include/whisper_mi355.h);
        beam search with compact drops finished windows' hypotheses from the passes.
        record_logprobs: per-step log-prob records in each GenResult.  stats: filled with the decode's counters."""
        W = len(slots)
        P = len(prompts[0])
        if any(len(p) != P for p in prompts):
            raise ValueError("all prompts of one generate call must have the same length")
        st = self.dims.specials
        if sot_index is None:
            sot_index = list(prompts[0]).index(st.sot) if st.sot in prompts[0] else -1
        h_slots = np.ascontiguousarray(slots, dtype=np.int32)
        h_prompts = np.ascontiguousarray(np.asarray(prompts, dtype=np.int32).reshape(W, P))
        sup = np.ascontiguousarray(sorted(set(int(t) for t in suppress_tokens)), dtype=np.int32)
        if sup.size == 0:
            sup = np.zeros(1, dtype=np.int32) - 1
        toks = np.zeros((W, max_length), dtype=np.int32)
        lens = np.zeros(W, dtype=np.int32)
        scores = np.zeros(W, dtype=np.float32)
        cum = np.zeros(W, dtype=np.float32)
        ns = np.zeros(W, dtype=np.float32)
        steps = np.zeros(1, dtype=np.int32)
        lp = np.full((W, max_length), np.nan, dtype=np.float32) if record_logprobs else None
        lpo = np.full((W, max_length), np.nan, dtype=np.float32) if record_logprobs else None
        st64 = np.zeros(4, dtype=np.int64)
        a = _capi.GenerateArgsC(
            W, _i32p(h_slots), P, _i32p(h_prompts), sot_index, beam_size, patience, length_penalty, max_length,
            temperature, num_hypotheses, seed, _i32p(sup), int(sup.size), int(bool(suppress_blank)),
            -1 if max_initial_timestamp_index is None else int(max_initial_timestamp_index), int(bool(with_timestamps)),
            check_every, _i32p(toks), _i32p(lens), _f32p(scores), _f32p(cum), _f32p(ns), _i32p(steps),
            int(max_rows), int(bool(compact)), _f32p(lp) if lp is not None else None,
            _f32p(lpo) if lpo is not None else None, st64.ctypes.data_as(C.POINTER(C.c_int64)))
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_generate(self.h, C.byref(a), self.stream_ptr()), "wm_generate")
        res = []
        for w in range(W):
            n = int(lens[w])
            r = GenResult(toks[w, :n].tolist(), float(scores[w]), float(cum[w]), float(ns[w]))
            if lp is not None:
                nr = min(max_length, n + (1 if P + n < max_length else 0))
                r.token_logprobs = lp[w, :nr].copy()
                r.token_logprobs_other = lpo[w, :nr].copy()
            res.append(r)
        if stats is not None:
            stats.update(passes=int(st64[0]), row_steps=int(st64[1]), refills=int(st64[2]), graph_captures=int(st64[3]))
        return res, int(steps[0])

    def forward(self, slots: Sequence[int], tokens: np.ndarray, last_only: bool = False,
                align_heads: Sequence[Tuple[int, int]] = ()) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Teacher-forced decoder forward. tokens [n_seq, S] -> logits [n_seq, S, V] (or [n_seq, V])."""
        tokens = np.ascontiguousarray(tokens, dtype=np.int32)
        n_seq, S = tokens.shape
        V = self.dims.n_vocab
        logits = torch.empty((n_seq, V) if last_only else (n_seq, S, V), device=self.device, dtype=torch.float32)
        h_slots = np.ascontiguousarray(slots, dtype=np.int32)
        na = len(align_heads)
        heads = np.ascontiguousarray(np.asarray(align_heads, dtype=np.int32).reshape(max(na, 1), 2) if na else np.zeros((1, 2), np.int32))
        attn = torch.empty((n_seq, S, na, self.dims.n_audio_ctx), device=self.device, dtype=torch.float32) if na else None
        if n_seq > self.n_hyp:
            self.reserve(max(self.n_slots, 1), n_seq)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_forward(self.h, n_seq, _i32p(h_slots), S, _i32p(tokens), C.c_void_p(logits.data_ptr()),
                                            int(last_only), _i32p(heads), na,
                                            C.c_void_p(attn.data_ptr()) if attn is not None else None,
                                            self.stream_ptr()), "wm_forward")
        return logits, attn

    def detect_language(self, slots: Sequence[int], lang_begin: int, n_langs: int) -> np.ndarray:
        """wm_detect_language: language-token probabilities [len(slots), n_langs] of one decoder step from
        <|startoftranscript|> per window (softmax on the device)."""
        h_slots = np.ascontiguousarray(slots, dtype=np.int32)
        probs = np.zeros((len(slots), n_langs), dtype=np.float32)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_detect_language(self.h, len(slots), _i32p(h_slots), lang_begin, n_langs, _f32p(probs),
                                                    self.stream_ptr()), "wm_detect_language")
        return probs

    def align(self, slot: int, sot_sequence: Sequence[int], text_tokens: Sequence[int], num_frames: int,
              alignment_heads: Sequence[Tuple[int, int]], median_filter_width: int = 7):
        """-> (text_token_probs [n_text], text_indices, time_indices) (CTranslate2 Whisper.align for one window)."""
        sot = np.ascontiguousarray(sot_sequence, dtype=np.int32)
        text = np.ascontiguousarray(text_tokens, dtype=np.int32)
        heads = np.ascontiguousarray(np.asarray(alignment_heads, dtype=np.int32).reshape(-1, 2))
        cap = len(text) + 1 + num_frames // 2 + 2
        probs = np.zeros(max(len(text), 1), dtype=np.float32)
        ti = np.zeros(cap, dtype=np.int32)
        tj = np.zeros(cap, dtype=np.int32)
        n = np.zeros(1, dtype=np.int32)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_align(self.h, slot, len(sot), _i32p(sot), len(text), _i32p(text), num_frames,
                                          _i32p(heads), heads.shape[0], median_filter_width, _f32p(probs), _i32p(ti),
                                          _i32p(tj), _i32p(n), self.stream_ptr()), "wm_align")
        k = int(n[0])
        return probs[: len(text)], ti[:k].copy(), tj[:k].copy()

    def align_batch(self, slots: Sequence[int], sot_sequence: Sequence[int], texts: Sequence[Sequence[int]],
                    num_frames: Sequence[int], alignment_heads: Sequence[Tuple[int, int]], median_filter_width: int = 7):
        """wm_align_batch: CTranslate2 Whisper.align for several windows at once -> one (text_token_probs,
        text_indices, time_indices) per window (every window needs >= 1 text token)."""
        n = len(slots)
        if n == 0:
            return []
        sot = np.ascontiguousarray(sot_sequence, dtype=np.int32)
        lens = [len(t) for t in texts]
        off = np.zeros(n + 1, dtype=np.int32)
        off[1:] = np.cumsum(lens)
        text = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.int32) for t in texts]), dtype=np.int32)
        nf = np.ascontiguousarray(num_frames, dtype=np.int32)
        cap = [l + 1 + f // 2 for l, f in zip(lens, nf)]
        poff = np.zeros(n, dtype=np.int64)
        poff[1:] = np.cumsum(cap)[:-1]
        heads = np.ascontiguousarray(np.asarray(alignment_heads, dtype=np.int32).reshape(-1, 2))
        probs = np.zeros(max(int(off[-1]), 1), dtype=np.float32)
        ti = np.zeros(sum(cap), dtype=np.int32)
        tj = np.zeros(sum(cap), dtype=np.int32)
        plen = np.zeros(n, dtype=np.int32)
        hs = np.ascontiguousarray(slots, dtype=np.int32)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_align_batch(self.h, n, _i32p(hs), len(sot), _i32p(sot), _i32p(off), _i32p(text), _i32p(nf),
                                                _i32p(heads), heads.shape[0], median_filter_width, _f32p(probs),
                                                poff.ctypes.data_as(C.POINTER(C.c_int64)), _i32p(ti), _i32p(tj),
                                                _i32p(plen), self.stream_ptr()), "wm_align_batch")
        out = []
        for i in range(n):
            a, k = int(poff[i]), int(plen[i])
            out.append((probs[off[i]: off[i + 1]].copy(), ti[a: a + k].copy(), tj[a: a + k].copy()))
        return out

    def dtw(self, cost: torch.Tensor):
        """DTW path of a device cost matrix [N, M] (f32)."""
        cost = cost.to(self.device, torch.float32).contiguous()
        N, M = cost.shape
        ti = np.zeros(N + M + 2, dtype=np.int32)
        tj = np.zeros(N + M + 2, dtype=np.int32)
        n = np.zeros(1, dtype=np.int32)
        with torch.cuda.device(self.device):
            _capi.check(self.lib.wm_dtw(self.h, C.c_void_p(cost.data_ptr()), N, M, _i32p(ti), _i32p(tj), _i32p(n),
                                        self.stream_ptr()), "wm_dtw")
        k = int(n[0])
        return ti[:k].copy(), tj[:k].copy()

