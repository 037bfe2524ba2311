#!/usr/bin/env python3
"""Throughput benchmark: Whisper transcription RTFx (audio-seconds per wall-second) on MI355X.

Workload (BASELINE.json config 4, per GPU): large-v3, bf16, greedy with timestamps, 150 x 30 s windows of the
seeded speech-like corpus per GPU (window-sharded: GPU r owns windows [150 r, 150 r + 150) of one long file;
weak scaling).  One "step" = the whole hot path over the GPU's 150 windows with the PCM already resident in
HBM: log-mel of the shard (+ the one-float global-max exchange between shards, the path's only cross-shard
value) -> clamp -> encoder -> cross-KV -> batched greedy decode with on-device timestamp rules -> host
segment split + detokenise + WebVTT string.  Weights are seeded random-init large-v3 weights (no checkpoints
offline) with a decisive, audio-dependent decoder program planted (vlog_amd/weights.py plant_margin: ~112 tokens
per window, segment boundaries every ~3.5 s), so the north_star parity gates can be checked on the bench's own
windows (the `parity` block); the JSON reports the actual tokens per window.

The default 1-GPU run appends a `variable` block to the same line: the realistic workload (plant margin_var: each
window's audio sets its transcript length, so windows end at different steps), 150 windows through the row-set
decode, timed the same way with its own roofline, decoder steps and active-row fraction (variable_block).

Prints ONE JSON line on rank 0.  `python bench.py` (N=1) or torch.distributed.run --nproc-per-node N.
"""
from __future__ import annotations

import argparse
from typing import Optional
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vlog_amd.audio import speech_like  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.segments import split_segments_by_timestamps  # noqa: E402
from vlog_amd.tokenizer import Tokenizer  # noqa: E402
from vlog_amd.vtt import generate_webvtt  # noqa: E402
from vlog_amd.weights import synthetic_state_dict  # noqa: E402

METRIC = "audio-sec transcribed per wall-sec (RTFx), large-v3, 1/2/4/8 MI355X; WER delta"
HBM_PEAK_GBS = 8000.0
MFMA_BF16_PEAK_TFS = 2500.0
# engine profile classes that are one kernel each (roofline candidates; see the dominant-class pick below)
SINGLE_KERNEL_CLASSES = ("cross_attn", "enc_attn", "self_attn", "logmel", "logits_gemm", "select", "crosskv_gemm")
CLIP = 480000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_shard(g0: int, W: int, cache=None, variable: bool = False):
    """PCM of windows [g0, g0 + W) of the corpus plus 200-sample margins from the neighbouring clips (window i is
    speech_like seed i; variable: the variable corpus, vlog_amd.audio.long_form_window, every 10th window room tone;
    `cache` maps seeds already generated to their clips)."""
    from vlog_amd.audio import long_form_window
    cache = {} if cache is None else cache

    def clip(i):
        if i not in cache:
            cache[i] = long_form_window(i) if variable else speech_like(30.0, i)
        return cache[i]
    clips = [clip(g0 + i) for i in range(W)]
    left = clip(g0 - 1)[-200:] if g0 > 0 else np.zeros(0, np.float32)
    right = clip(g0 + W)[:200]
    return np.concatenate([left] + clips + [right]).astype(np.float32), len(left)


class Pipeline:
    def __init__(self, eng, tok, dims, rank, world, W, beam, pcm_dev, margin_left, n_total, host_group=None,
                 words: bool = False, check_every: int = 4, g0: Optional[int] = None, max_rows: int = -1):
        """max_rows: -1 decodes every window in one all-rows batch; >= 0 runs the row-set decode (wm_generate
        max_rows, 0 = all windows at once) with the windows ordered longest-expected first and compaction."""
        self.eng, self.tok, self.dims = eng, tok, dims
        self.g0 = rank * W if g0 is None else g0       # first corpus window of this shard
        self.max_rows = max_rows
        self.check_every = check_every
        self.words = words
        if words:
            # the product's word-timestamp glue (WhisperModel.add_word_timestamps / find_alignment: one batched
            # wm_align_batch over every window with text), bound to this engine
            import functools
            import types
            from vlog_amd.transcribe import FRAMES_PER_SECOND, TOKENS_PER_SECOND, WhisperModel
            m = types.SimpleNamespace(engine=eng, dims=dims, frames_per_second=FRAMES_PER_SECOND,
                                      tokens_per_second=TOKENS_PER_SECOND)
            m.find_alignment = functools.partial(WhisperModel.find_alignment, m)
            self._add_words = functools.partial(WhisperModel.add_word_timestamps, m)
        self.host_group = host_group
        self.keep_windows = ()                  # windows whose encoder output the next step copies to the host
        self.rank, self.world, self.W, self.beam = rank, world, W, beam
        self.pcm_dev, self.margin_left, self.n_total = pcm_dev, margin_left, n_total
        st = dims.specials
        self.prompt = [st.sot, st.lang_token("en"), st.transcribe]
        self.suppress = list(tok.suppressed_tokens([-1]))
        self.stage = {}
        self.solo = False          # True: this rank steps alone (no cross-rank exchange)
        self.last_gmax = None

    def step(self):
        eng, W, d = self.eng, self.W, self.dims
        t0 = time.perf_counter()
        frame0 = self.g0 * 3000
        mel, gmax = eng.logmel(self.pcm_dev, n_samples=self.n_total, pcm_offset=frame0 * 160 - self.margin_left,
                               frame0=frame0, n_frames=W * 3000)
        if self.world > 1 and self.solo:
            # a step on one rank alone (the untimed parity leg): the other ranks are not in the exchange, so
            # reuse the whole-file max of the last exchanged step (same PCM, same value)
            if self.last_gmax is None:
                raise RuntimeError("solo step before any exchanged step: no whole-file log-mel max to reuse")
            eng.logmel_finalize(mel, gmax, self.last_gmax)
        elif self.world > 1:
            # faster-whisper's clamp uses the WHOLE file's log-mel max: the one cross-shard value, exchanged
            # as a host float over a gloo group (no RCCL collective on the data path)
            import torch.distributed as dist
            g = torch.tensor([eng.gmax_value(gmax)], dtype=torch.float32)
            dist.all_reduce(g, op=dist.ReduceOp.MAX, group=self.host_group)
            self.last_gmax = float(g[0])
            eng.logmel_finalize(mel, gmax, self.last_gmax)
        else:
            eng.logmel_finalize(mel, gmax)          # single shard: the clamp reads the max on the device
        t1 = time.perf_counter()
        enc = eng.encode(mel, [i * 3000 for i in range(W)], [3000] * W)
        eng.cross_kv(enc, 0)
        torch.cuda.synchronize(eng.device)
        t2 = time.perf_counter()
        gen_stats = {}
        if self.max_rows >= 0 and self.beam == 1:
            # row-set decode: expected tokens from the shard's frame energy (the VAD stand-in's GPU kernel), windows
            # started longest-expected first, finished rows refilled / compacted (vlog_amd/shard.py, engine.cpp)
            from vlog_amd.shard import expected_token_order, expected_tokens
            db = eng.frame_energy_db(self.pcm_dev, 512)
            exp = expected_tokens(db, 512, [self.margin_left + CLIP * i for i in range(W)], [CLIP] * W)
            order = expected_token_order(exp)
            out, steps = eng.generate(order, [self.prompt] * W, suppress_tokens=self.suppress, max_length=448,
                                      check_every=self.check_every, max_rows=self.max_rows, compact=True,
                                      stats=gen_stats)
            res = [None] * W
            for w, r in zip(order, out):
                res[w] = r
        else:
            # beam: with the row-set option, finished windows' hypotheses leave the passes (beam compaction)
            res, steps = eng.generate(list(range(W)), [self.prompt] * W, beam_size=self.beam,
                                      suppress_tokens=self.suppress, max_length=448, check_every=self.check_every,
                                      compact=self.max_rows >= 0, stats=gen_stats)
        t3 = time.perf_counter()
        groups = []
        for w, r in enumerate(res):
            off = (self.g0 + w) * 30.0
            cur, _, _ = split_segments_by_timestamps(r.tokens, d.specials.timestamp_begin, off, 3000, 30.0, w * 3000)
            groups.append(cur)
        t_al = 0.0
        if self.words:
            ta = time.perf_counter()
            idx = [w for w, g in enumerate(groups) if g]
            if idx:
                self._add_words([groups[w] for w in idx], self.tok, [3000] * len(idx), "\"'“¿([{-",
                                "\"'.。,，!！?？:：”)]}、", 0.0, slots=idx)
            t_al = time.perf_counter() - ta
        segs = []
        for cur in groups:
            for s in cur:
                text = self.tok.decode(s["tokens"])
                if s["start"] == s["end"] or not text.strip():
                    continue
                segs.append({"start": s["start"], "end": s["end"], "text": text})
        vtt = generate_webvtt(segs)
        t4 = time.perf_counter()
        for k, v in (("logmel", t1 - t0), ("encode", t2 - t1), ("decode", t3 - t2), ("align", t_al),
                     ("host", t4 - t3 - t_al)):
            self.stage[k] = self.stage.get(k, 0.0) + v
        import zlib
        crc = 0
        for r in res:
            crc = zlib.crc32(np.asarray(r.tokens, dtype=np.int32).tobytes(), crc)
        self.last = dict(tokens=[len(r.tokens) for r in res], steps=steps, segments=len(segs), vtt_bytes=len(vtt),
                         crc=crc, gen_stats=gen_stats)
        if self.keep_windows:
            self.kept = dict(res=res, enc={w: enc[w].float().cpu().numpy() for w in self.keep_windows})
        del enc, mel

    def run_stream(self, K: int):
        """K batches of this shard's W windows through ONE continuous row-set decode: every batch's log-mel +
        encoder output goes to its own window slots (K x W slots), then the windows of all K batches decode with W
        rows in flight, longest-expected first, a finished window's row taking the next window (engine.cpp
        generate_rows) — so a batch's short windows no longer wait for its longest one: the decoder steps follow the
        total tokens, plus one tail at the end.  A production worker streaming its shard does the same.  Beam search:
        W windows' groups of `beam` rows in flight (engine.cpp generate_rows_beam); word timestamps: one batched
        alignment over every window at the end.  Results, segments and the WebVTT are produced for every window of
        every batch."""
        from vlog_amd.shard import expected_token_order, expected_tokens
        eng, W, d = self.eng, self.W, self.dims
        t0 = time.perf_counter()
        frame0 = self.g0 * 3000
        t_mel = t_enc = 0.0
        for k in range(K):
            ta = time.perf_counter()
            mel, gmax = eng.logmel(self.pcm_dev, n_samples=self.n_total, pcm_offset=frame0 * 160 - self.margin_left,
                                   frame0=frame0, n_frames=W * 3000)
            if self.world > 1:
                import torch.distributed as dist
                g = torch.tensor([eng.gmax_value(gmax)], dtype=torch.float32)
                dist.all_reduce(g, op=dist.ReduceOp.MAX, group=self.host_group)
                self.last_gmax = float(g[0])
                eng.logmel_finalize(mel, gmax, self.last_gmax)
            else:
                eng.logmel_finalize(mel, gmax)
            tb = time.perf_counter()
            enc = eng.encode(mel, [i * 3000 for i in range(W)], [3000] * W)
            eng.cross_kv(enc, k * W)
            del enc, mel
            torch.cuda.synchronize(eng.device)
            tc = time.perf_counter()
            t_mel += tb - ta
            t_enc += tc - tb
        t2 = time.perf_counter()
        db = eng.frame_energy_db(self.pcm_dev, 512)
        exp = expected_tokens(db, 512, [self.margin_left + CLIP * i for i in range(W)], [CLIP] * W)
        order = expected_token_order(np.tile(exp, K))
        gen_stats = {}
        # beam search: W windows' groups of `beam` rows in flight (engine.cpp generate_rows_beam)
        kw = dict(beam_size=self.beam, patience=1.0) if self.beam > 1 else {}
        out, steps = eng.generate(order, [self.prompt] * (K * W), suppress_tokens=self.suppress, max_length=448,
                                  check_every=self.check_every, max_rows=W * max(1, self.beam), compact=True,
                                  stats=gen_stats, **kw)
        res = [None] * (K * W)
        for w, r in zip(order, out):
            res[w] = r
        t3 = time.perf_counter()
        groups = []
        for k in range(K):
            for w in range(W):
                off = (self.g0 + w) * 30.0
                cur, _, _ = split_segments_by_timestamps(res[k * W + w].tokens, d.specials.timestamp_begin, off, 3000,
                                                         30.0, w * 3000)
                groups.append(cur)
        t_al = 0.0
        if self.words:
            # every window's encoder output is still in its slot (k W + w): one batched alignment over all of them
            ta = time.perf_counter()
            idx = [i for i, g in enumerate(groups) if g]
            if idx:
                self._add_words([groups[i] for i in idx], self.tok, [3000] * len(idx), "\"'“¿([{-",
                                "\"'.。,，!！?？:：”)]}、", 0.0, slots=idx)
            t_al = time.perf_counter() - ta
        n_seg = vtt_bytes = 0
        for k in range(K):
            segs = []
            for w in range(W):
                cur = groups[k * W + w]
                for s_ in cur:
                    text = self.tok.decode(s_["tokens"])
                    if s_["start"] == s_["end"] or not text.strip():
                        continue
                    segs.append({"start": s_["start"], "end": s_["end"], "text": text})
            vtt = generate_webvtt(segs)
            n_seg += len(segs)
            vtt_bytes += len(vtt)
        t4 = time.perf_counter()
        for k_, v in (("logmel", t_mel), ("encode", t_enc), ("schedule", 0.0), ("decode", t3 - t2), ("align", t_al),
                      ("host", t4 - t3 - t_al)):
            self.stage[k_] = self.stage.get(k_, 0.0) + v
        import zlib
        crc = 0
        for r in res[:W]:
            crc = zlib.crc32(np.asarray(r.tokens, dtype=np.int32).tobytes(), crc)
        self.last = dict(tokens=[len(r.tokens) for r in res[:W]], steps=steps / K, segments=n_seg, vtt_bytes=vtt_bytes,
                         crc=crc, gen_stats=gen_stats, stream_batches=K,
                         all_tokens=[len(r.tokens) for r in res])
        return time.perf_counter() - t0


def host_cpu() -> dict:
    """lscpu model name and physical core count of this host (the CPU baseline states both)."""
    info = {"model": None, "physical_cores": None, "logical_cpus": os.cpu_count()}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name")
        if kv.get("Core(s) per socket") and kv.get("Socket(s)"):
            info["physical_cores"] = int(kv["Core(s) per socket"]) * int(kv["Socket(s)"])
    except Exception:
        pass
    if info["model"] is None and os.path.isfile("/proc/cpuinfo"):
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    info["cpu_share"] = cpu_share()
    return info


def cpu_share() -> int:
    """CPUs this process may actually use: the affinity mask, capped by the cgroup-v2 CPU quota (a GPU box grants
    one process a share of the host, far fewer CPUs than `os.cpu_count()` reports)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def composite_roofline(dims, lengths, steps: int, prompt_len: int, elapsed_per_step: float, windows: int) -> dict:
    """SURVEY.md §8(d) composite bound for one step: encoder FLOPs at the dense bf16 MFMA peak plus decoder bytes at
    the HBM peak, over the measured step time, using the ACTUAL generated length of every window.  Two byte
    accountings: `factored` (what this engine streams: each active window's encoder output, L x 1500 x d bf16,
    per decoder step) and `projected` (§8(d) as written: L x 2 x 1500 x d bf16 of cross-K/V per window-step,
    plus the K/V projection FLOPs)."""
    L, d, T = dims.n_dec_layer, dims.n_state, dims.n_audio_ctx
    win_steps = sum(n + 1 for n in lengths)                        # token-producing steps per window (incl. eot)
    pos_sum = sum(sum(prompt_len + s for s in range(n + 1)) for n in lengths)
    w_bytes = dims.decoder_weight_bytes() * steps
    self_kv = dims.self_kv_bytes_per_position() * pos_sum
    enc_fl = dims.encoder_flops_per_window() * windows
    out = {}
    for name, xbytes, xfl in (("factored", L * T * d * 2.0, 0.0),
                              ("projected", dims.cross_kv_bytes_per_window(), dims.cross_kv_flops_per_window())):
        t_mfma = (enc_fl + xfl * windows) / (MFMA_BF16_PEAK_TFS * 1e12)
        t_hbm = (w_bytes + self_kv + xbytes * win_steps) / (HBM_PEAK_GBS * 1e9)
        out[name] = {"t_ideal_ms": round(1e3 * (t_mfma + t_hbm), 2), "mfma_ms": round(1e3 * t_mfma, 2),
                     "hbm_ms": round(1e3 * t_hbm, 2), "frac": round((t_mfma + t_hbm) / elapsed_per_step, 4)}
    return out


def parity_sample(dims, sd, pipe, fp8_cross: bool = False) -> dict:
    """Outside the timed region: the north_star gates (tests/parity_util.py gate_windows) on sampled windows of
    the last step: every GPU token sequence teacher-forced through the CPU oracle (engine numeric format) from
    the GPU's own encoder output (identical = the GPU token is the oracle's argmax at every step, so the oracle's
    greedy search yields the same sequence); non-identical windows re-decoded by the oracle's greedy search
    for the WER delta (GPU text vs oracle text; no ground truth exists for synthetic audio) and the segment
    times.  With --cross-fp8 the oracle sees the full-precision encoder output: the fp8 mode is gated against
    bf16 arithmetic, not against itself."""
    sys.path.insert(0, ROOT)
    from oracle.decode import GenerateOptions
    from oracle.model import OracleWhisper
    from tests.parity_util import gate_windows
    from vlog_amd.weights import round_bf16

    orc = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)
    res, enc = pipe.kept["res"], pipe.kept["enc"]
    opt = GenerateOptions(suppress_tokens=pipe.suppress, max_length=448)
    ws = sorted(enc)
    g = gate_windows(orc, lambda w: np.stack([enc[i] for i in w]), pipe.prompt, res, dims.specials, opt, pipe.tok,
                     windows=ws, time_offset=lambda w: (pipe.g0 + w) * 30.0)
    g.pop("oracle_tokens")
    g["windows"] = ws
    g["method"] = ("every sampled window's GPU tokens teacher-forced through oracle/ (bf16-activation mode) on the "
                   "GPU's encoder output; identical = the GPU token is the oracle's argmax at every step; "
                   "wer_delta = WER of the GPU text vs the oracle's greedy text; segment times split from both "
                   "token streams (tests/parity_util.py gate_windows)")
    return g


def cpu_baseline(dims, sd, mean_tokens: float, n_positions: int = 4):
    """Oracle (numpy fp32, this repo's CPU restatement) on the host cores: one 30 s window's log-mel + encoder +
    cross-KV, plus single greedy decoder steps timed at `n_positions` positions spread over the window's mean token
    count (each after a teacher-forced prefill of the tokens before it, untimed), so the per-step cost covers the
    growing self-attention; extrapolated to the GPU run's mean tokens per window."""
    sys.path.insert(0, ROOT)
    from oracle import mel as omel
    from oracle.model import OracleWhisper
    from vlog_amd.weights import round_bf16

    st = dims.specials
    # every CPU this process is granted (all cores): numpy's BLAS threads follow the thread pool size
    share = cpu_share()
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=share)
    except ImportError:
        limiter = None
    orc = OracleWhisper(round_bf16(sd), dims, np.float32)
    x = speech_like(30.0, 0)
    t0 = time.perf_counter()
    f = omel.log_mel(x, dims.n_mels)
    enc = orc.encode(omel.pad_or_trim(f)[None])
    cross = orc.cross_kv(enc)
    t1 = time.perf_counter()
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    n_tok = max(1, int(round(mean_tokens)))
    positions = sorted({int(round(i * (n_tok - 1) / max(1, n_positions - 1))) for i in range(n_positions)})
    rng = np.random.default_rng(0)
    step_s = []
    for p in positions:
        toks = prompt + [int(t) for t in rng.integers(1000, st.eot - 1000, size=p)]      # any text history
        _, cache = orc.decode(np.asarray([toks]), cross)
        ts = time.perf_counter()
        logits, _ = orc.decode(np.asarray([[toks[-1]]]), cross, cache=cache, offset=len(toks))
        int(np.argmax(logits[0, -1]))                                                    # the greedy pick
        step_s.append(time.perf_counter() - ts)
    per_step = float(np.mean(step_s))
    per_window = (t1 - t0) + per_step * (n_tok + 1)
    threads = share
    if limiter is not None:
        from threadpoolctl import threadpool_info
        threads = max([p.get("num_threads", 0) for p in threadpool_info()] + [1])
        limiter.unregister()
    hc = host_cpu()
    return {"value": round(30.0 / per_window, 4), "unit": "audio_s/s", "cores": threads, "kind": "port",
            "cpu_model": hc["model"], "host_physical_cores": hc["physical_cores"], "host_logical_cpus": hc["logical_cpus"],
            "process_cpu_share": hc["cpu_share"],
            "sample": (f"oracle/ numpy fp32 CPU restatement, {dims.name}: one 30 s window log-mel+encoder+cross-KV "
                       f"({t1 - t0:.1f} s) + greedy decoder steps timed at positions {positions} "
                       f"({', '.join(f'{1e3 * v:.0f}' for v in step_s)} ms), mean {per_step:.3f} s/step, extrapolated "
                       f"to {mean_tokens:.1f} tokens + <|endoftext|> per window; faster-whisper CPU baseline "
                       f"unavailable (not installed)")}


def roofline_block(breakdown, prof, dom, args, beam: int = 1, traffic_json: Optional[str] = None) -> dict:
    """kernels_one_step, roofline (the dominant single-kernel class over the timed region), encoder_mfma and
    decoder_kv_read from the engine's event profiler."""
    out = {}
    kern = {}
    for k, v in breakdown.items():
        if v["launches"] == 0:
            continue
        kern[k] = {"launches": v["launches"], "ms": round(v["ms"], 3),
                   "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2) if v["flops"] else None,
                   "gbs": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["bytes"] else None}
    out["kernels_one_step"] = kern
    v = prof[dom]                          # measured over the timed region
    if dom in ("cross_attn", "self_attn", "select", "dec_other", "logmel") or (v["flops"] == 0):
        ach = v["bytes"] / (v["ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4)}
    else:
        ach = v["flops"] / (v["ms"] * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": MFMA_BF16_PEAK_TFS, "unit": "TFLOP/s",
                "frac": round(ach / MFMA_BF16_PEAK_TFS, 4)}
    roof["kernel"] = dom
    roof["launches"] = v["launches"]
    roof["avg_launch_us"] = round(1000.0 * v["ms"] / max(v["launches"], 1), 2)
    roof["traffic"] = None
    tj_path = args.traffic_json if traffic_json is None else traffic_json
    if tj_path and os.path.isfile(tj_path):
        try:
            tj = json.load(open(tj_path))
            roof["traffic"] = tj.get(dom)
            if roof["traffic"] is not None:
                # not measured in this run: PMC counters need their own rocprofv3 passes (tools/pmc_traffic.sh)
                roof["traffic_source"] = (f"{os.path.relpath(tj_path, ROOT)}: committed rocprofv3 --pmc passes "
                                          "(FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) of this kernel on this "
                                          "workload; HBM bytes per launch, not measured in this run")
        except Exception:
            pass
    if beam > 1 and not args.cross_fp8:
        roof["accounting"] = ("projected cross-attention (beam groups): algorithmic bytes = each active window's "
                              "K and V panels (L x 2 x 1500 x d bf16) per launch, counted in-kernel")
    else:
        roof["accounting"] = ("factored cross-attention: algorithmic bytes = each active window's encoder output "
                              + ("(L x 1500 x d e4m3 + 1500 f32 scales)" if args.cross_fp8 else "(L x 1500 x d bf16)")
                              + " + q' per launch, counted in-kernel")
    out["roofline"] = roof
    enc_ms = sum(breakdown[k]["ms"] for k in ("enc_gemm", "enc_attn", "crosskv_gemm"))
    enc_fl = sum(breakdown[k]["flops"] for k in ("enc_gemm", "enc_attn", "crosskv_gemm"))
    out["encoder_mfma"] = {"achieved_tflops": round(enc_fl / max(enc_ms, 1e-9) / 1e9, 1),
                           "frac_of_2500": round(enc_fl / max(enc_ms, 1e-9) / 1e9 / MFMA_BF16_PEAK_TFS, 4)}
    cx = breakdown["cross_attn"]
    out["decoder_kv_read"] = {"achieved_gbs": round(cx["bytes"] / max(cx["ms"], 1e-9) / 1e6, 1),
                              "frac_of_8000": round(cx["bytes"] / max(cx["ms"], 1e-9) / 1e6 / HBM_PEAK_GBS, 4)}
    return out


def timed_run(pipe, eng, steps: int, warmup: int, barrier, profile: bool = True, stream: bool = False):
    """W untimed warmup steps, one untimed step with every kernel class under events (the breakdown and the
    dominant single-kernel class), then exactly `steps` timed steps (events on the dominant class only), bracketed
    by the barrier.  -> (elapsed s, breakdown, timed-region profile, dominant class, stage times of the timed steps)"""
    for _ in range(warmup):
        pipe.step()
    breakdown, dom = None, None
    if profile:
        barrier()
        eng.profile(True)
        pipe.step()
        eng.profile(False)
        breakdown = eng.profile_read()
        # the roofline names ONE kernel (it must match one rocprof row): classes that group several kernel
        # variants (the GEMM families, combines, misc) are not candidates.  Events around the 27k decoder-GEMM
        # launches per step would also slow the timed region.
        single = {k: v for k, v in breakdown.items() if k in SINGLE_KERNEL_CLASSES and v["launches"]}
        dom = max(single or breakdown, key=lambda k: (single or breakdown)[k]["ms"])
    pipe.stage = {}
    barrier()
    if dom is not None:                       # timed region: events on the dominant class only
        eng.profile(True, classes=[dom])
    t0 = time.perf_counter()
    if stream:
        pipe.run_stream(steps)
    else:
        for _ in range(steps):
            pipe.step()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = None
    if dom is not None:
        eng.profile(False)
        prof = eng.profile_read()
    return elapsed, breakdown, prof, dom, dict(pipe.stage)


def variable_block(args, dims, base_sd, tok, local: int, steps: int, warmup: int = 1) -> dict:
    """The realistic workload in the same run: the margin_var plant (a window's audio sets where
    its script ends, so windows decode different numbers of tokens), 150 windows of the same corpus, the row-set
    decode (max_rows 0: all windows in flight, longest-expected first, finished rows compacted) -- the product's
    throughput-mode schedule.  Timed exactly like the headline, on a fresh engine; no parity sample (the variable
    gates run in tests/test_gpu_gates.py)."""
    from vlog_amd.engine import GpuEngine
    from vlog_amd.weights import plant_margin
    t = time.perf_counter()
    plant_margin(base_sd, dims, 0, variable=True)
    eng = GpuEngine(dims, base_sd, local)
    W = args.windows
    pcm, margin = build_shard(0, W, variable=True)
    pcm_dev = torch.from_numpy(pcm).to(eng.device)
    eng.reserve(W, W)
    pipe = Pipeline(eng, tok, dims, 0, 1, W, 1, pcm_dev, margin, W * CLIP, None, check_every=args.check_every,
                    g0=0, max_rows=0)
    setup = time.perf_counter() - t
    elapsed, breakdown, prof, dom, stage = timed_run(pipe, eng, steps, warmup, lambda: torch.cuda.synchronize(eng.device),
                                                     profile=not args.no_profile)
    toks = pipe.last["tokens"]
    gs = pipe.last["gen_stats"]
    blk = {"workload": "variable (weights.py plant margin_var; row-set decode, max_rows 0, longest-expected first, "
                       "compaction)",
           "value": round(W * 30.0 * steps / elapsed, 2), "unit": "audio_s/s", "steps": steps, "warmup": warmup,
           "ms_per_step": round(1000 * elapsed / steps, 2), "windows": W, "setup_s": round(setup, 1),
           "mean_tokens_per_window": round(float(np.mean(toks)), 1),
           "token_length_min_p50_max": [int(np.min(toks)), int(np.median(toks)), int(np.max(toks))],
           "decoder_steps": pipe.last["steps"], "decoder_row_steps": gs.get("row_steps"),
           "decoder_passes": gs.get("passes"),
           "active_row_fraction": (round(sum(n + 1 for n in toks) / gs["row_steps"], 4) if gs.get("row_steps") else None),
           "token_crc32": pipe.last["crc"],
           "stages_s_per_step": {k: round(v / steps, 4) for k, v in stage.items()}}
    if prof:
        rb = roofline_block(breakdown, prof, dom, args, traffic_json="")
        blk["roofline"] = rb["roofline"]
        blk["encoder_mfma"] = rb["encoder_mfma"]
        blk["decoder_kv_read"] = rb["decoder_kv_read"]
        blk["kernels_one_step"] = rb["kernels_one_step"]
    blk.setdefault("roofline", {})["composite"] = composite_roofline(dims, toks, pipe.last["steps"], len(pipe.prompt),
                                                                   elapsed / steps, W)
    del pipe, eng, pcm_dev
    torch.cuda.empty_cache()
    return blk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--windows", type=int, default=150, help="30 s windows per GPU")
    ap.add_argument("--beam", type=int, default=1)
    ap.add_argument("--word-timestamps", action="store_true", help="config 5: batched word alignment in every step")
    ap.add_argument("--eot-after", type=int, default=110, help="with --random-weights: the planted EOT position")
    ap.add_argument("--random-weights", action="store_true",
                    help="plain random-init weights + planted EOT (round-2 workload) instead of the margin-planted "
                         "model; same kernels and token counts, but near-tied logits (the parity gates cannot hold)")
    ap.add_argument("--check-every", type=int, default=4, help="decode steps between host polls of the live count")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=None, help="PMC traffic summary (default: profiles/traffic_r06_b.json, "
                    "or traffic_r02_fp8.json with --cross-fp8)")
    ap.add_argument("--cross-fp8", action="store_true", help="opt-in fp8 (e4m3) cross memory: not the headline")
    ap.add_argument("--no-profile", action="store_true", help="skip the live per-kernel event timing")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle parity sample (rank 0, untimed)")
    ap.add_argument("--parity-windows", type=int, default=16)
    ap.add_argument("--workload", choices=("uniform", "variable"), default="uniform",
                    help="uniform: the margin-planted model (every window ~112 tokens); variable: plant margin_var on "
                         "the variable corpus (a window's audio level sets where its script ends: 44 to ~225 tokens "
                         "for speech, one token for the room-tone window in every 10)")
    ap.add_argument("--max-rows", type=int, default=None,
                    help="row-set decode with at most this many rows in flight (0 = all windows at once), windows "
                         "ordered longest-expected first, finished rows refilled / compacted; -1 = one all-rows "
                         "batch.  Default: -1 for the uniform workload, 0 for the variable one")
    ap.add_argument("--stream", action="store_true",
                    help="the --steps batches of the shard through ONE continuous row-set decode (Pipeline.run_stream): "
                         "finished windows' rows refilled from the next batch; ms_per_step = total / steps")
    ap.add_argument("--balance", choices=("count", "tokens"), default=None,
                    help="N > 1: windows per GPU by count, or by expected tokens (default for --workload variable)")
    ap.add_argument("--no-variable", action="store_true",
                    help="skip the variable-length block the default (uniform, 1 GPU) run appends to its line")
    ap.add_argument("--variable-steps", type=int, default=None, help="timed steps of the variable block (default "
                    "max(2, steps // 4))")
    args = ap.parse_args()
    if args.max_rows is None:
        args.max_rows = 0 if args.workload == "variable" else -1
    if args.balance is None:
        args.balance = "tokens" if args.workload == "variable" else "count"
    if args.traffic_json is None:
        # the committed PMC files were measured on the default workload (uniform greedy, 150 windows); another
        # workload's launches move other bytes, so its line carries traffic null unless a file is given
        args.traffic_json = (os.path.join(ROOT, "profiles", "traffic_r02_fp8.json" if args.cross_fp8 else "traffic_r06_b.json")
                             if args.beam == 1 and args.workload == "uniform" and args.windows == 150 else "")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VLOG_AMD_BENCH_SHARE_GPU=1: a rehearsal of the N > 1 path with every rank on
    # the visible GPUs round-robin (RCCL refuses two ranks on one device; no collective is on the data path)
    if os.environ.get("VLOG_AMD_BENCH_SHARE_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    host_group = None
    json_fd = None
    if world > 1:
        # the process-group backends print connection notices on stdout ("[Gloo] Rank ..."); the driver reads ONE
        # JSON line from rank 0, so fd 1 goes to stderr for the run and the line is written to the saved stdout
        sys.stdout.flush()
        json_fd = os.dup(1)
        os.dup2(2, 1)
        import torch.distributed as dist
        # one gloo process group for the host scalars (log-mel max, expected-token estimates, timing): the windows
        # shard with no device collective, so RCCL is never brought up; each rank's GPU comes from
        # LOCAL_RANK (torch.cuda.set_device above)
        dist.init_process_group("gloo")
        host_group = dist.group.WORLD

    dims = model_dims(args.model)
    t = time.perf_counter()
    plant = "margin_var" if args.workload == "variable" else "margin"
    # the default 1-GPU line also times the variable-length workload (variable_block) on a second engine
    run_var = (world == 1 and args.workload == "uniform" and args.beam == 1 and not args.stream and not args.cross_fp8
               and not args.random_weights and not args.no_variable and args.max_rows < 0 and dims.n_dec_layer >= 4)
    base_sd = None
    if args.random_weights:
        sd = synthetic_state_dict(dims, seed=0, eot_after=args.eot_after)
    elif run_var:
        # one seeded random-init draw, planted twice (per-tensor generators: identical to generating each plant)
        from vlog_amd.weights import plant_margin
        base_sd = synthetic_state_dict(dims, seed=0)
        sd = {k: v.clone() for k, v in base_sd.items()}
        plant_margin(sd, dims, 0, variable=False)
    else:
        sd = synthetic_state_dict(dims, seed=0, plant=plant)
    from vlog_amd.engine import GpuEngine
    eng = GpuEngine(dims, sd, local)
    if args.cross_fp8:
        eng.set_option("cross_fp8", 1)
    if args.beam > 1 and not args.cross_fp8:
        eng.set_option("cross_mode", 0)        # the product's choice for beam groups (transcribe.py decode_windows)
    keep_sd = rank == 0 and ((world == 1 and not args.no_cpu_baseline) or not args.no_parity)
    if not keep_sd:
        del sd
        sd = None
    tok = Tokenizer(dims, language="en")
    W_nat = W = args.windows
    g0 = rank * W
    cache = {}
    var_corpus = args.workload == "variable"
    pcm, margin = build_shard(g0, W, cache, variable=var_corpus)
    if world > 1 and args.balance == "tokens":
        # work-balanced shards (vlog_amd/shard.py): every rank estimates the expected tokens of its natural window
        # range from the GPU frame energy, the estimates are exchanged as host floats, and the corpus is re-cut into
        # contiguous ranges of equal expected tokens (setup, untimed; a coordinator does the same before dispatch)
        import torch.distributed as dist
        from vlog_amd.shard import expected_tokens, partition_by_weight
        db = eng.frame_energy_db(torch.from_numpy(pcm), 512)
        est = torch.tensor(expected_tokens(db, 512, [margin + CLIP * i for i in range(W)], [CLIP] * W), dtype=torch.float64)
        parts = [torch.zeros_like(est) for _ in range(world)]
        dist.all_gather(parts, est, group=host_group)
        g0, g1 = partition_by_weight(torch.cat(parts).numpy(), world)[rank]
        W = g1 - g0
        pcm, margin = build_shard(g0, W, cache, variable=var_corpus)
    del cache
    pcm_dev = torch.from_numpy(pcm).to(eng.device)
    n_total = world * W_nat * CLIP
    eng.reserve(W * (args.steps if args.stream else 1), W * max(1, args.beam))
    log(f"[rank {rank}] setup {time.perf_counter() - t:.1f} s, windows [{g0}, {g0 + W}), engine "
        f"{eng.device_bytes() / 2**30:.1f} GiB")
    pipe = Pipeline(eng, tok, dims, rank, world, W, args.beam, pcm_dev, margin, n_total, host_group,
                    words=args.word_timestamps, check_every=args.check_every, g0=g0, max_rows=args.max_rows)

    def barrier():
        # device drained, then a host-side rendezvous over the gloo group: no RCCL call anywhere in the timed
        # region
        torch.cuda.synchronize(eng.device)
        if world > 1:
            import torch.distributed as dist
            dist.barrier(group=host_group)

    elapsed, breakdown, prof, dom, stage_timed = timed_run(pipe, eng, args.steps, args.warmup, barrier,
                                                           profile=not args.no_profile, stream=args.stream)
    rank_info = [[elapsed, W, float(sum(pipe.last.get("all_tokens", pipe.last["tokens"]))), pipe.last["steps"]]]
    if world > 1:
        import torch.distributed as dist
        te = torch.tensor(rank_info[0], dtype=torch.float64)
        parts = [torch.zeros_like(te) for _ in range(world)]
        dist.all_gather(parts, te, group=host_group)
        rank_info = [p.tolist() for p in parts]
        elapsed = max(r[0] for r in rank_info)             # the job ends with its slowest rank
    parity = None
    if rank == 0 and not args.no_parity and sd is not None and args.beam == 1:
        from tests.parity_util import sample_indices
        pipe.keep_windows = tuple(sample_indices(W, args.parity_windows))
        pipe.solo = True                                        # rank 0 alone: no exchange with the other ranks
        pipe.step()                                             # untimed: keeps the sampled windows' encoder output
        try:
            parity = parity_sample(dims, sd, pipe, fp8_cross=args.cross_fp8)
        except Exception as e:  # reported, never fatal to the GPU measurement
            parity = {"error": str(e)[:300]}
    audio_s = world * W_nat * 30.0 * args.steps           # every rank's windows (balanced shards sum to the same)
    value = audio_s / elapsed
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    toks = pipe.last["tokens"]
    mean_tok = float(np.mean(toks))
    # BASELINE.json configs: 4 = large-v3 bf16 greedy (the headline), 5 = large-v3 beam 5 + word timestamps
    cfg_name = ("config 4" if args.beam == 1 and not args.word_timestamps and args.model == "large-v3" else
                "config 5" if args.beam > 1 and args.word_timestamps and args.model == "large-v3" else "non-config variant")
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "audio_s/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16+e4m3-cross" if args.cross_fp8 else "bf16",
        "data": "synthetic",
        "config": {"workload": f"{cfg_name}: {args.model} bf16{' (opt-in fp8 e4m3 cross memory)' if args.cross_fp8 else ''} "
                               f"{'greedy' if args.beam == 1 else 'beam_size=%d' % args.beam}"
                               f"{' + word_timestamps' if args.word_timestamps else ''}, timestamps on, "
                               f"{W} x 30 s windows per GPU of the seeded speech-like corpus "
                               f"({args.workload} transcript lengths), window-sharded",
                   "model": args.model, "windows_per_gpu": W, "audio_s_per_gpu_per_step": W * 30.0,
                   "mean_tokens_per_window": round(mean_tok, 1), "decoder_steps": pipe.last["steps"],
                   "token_length_min_p50_max": [int(np.min(toks)), int(np.median(toks)), int(np.max(toks))],
                   "decode": (f"continuous row-set over the {args.steps} batches "
                              f"({W} windows in flight{' x %d beam rows' % args.beam if args.beam > 1 else ''}, "
                              f"longest-expected first, refill across batches + compaction)" if args.stream else
                              "all-rows batch" if args.max_rows < 0 else
                              f"row-set (max_rows {args.max_rows or W}, longest-expected first, refill + compaction)"),
                   "decoder_row_steps": pipe.last["gen_stats"].get("row_steps"),
                   # live rows / rows in the passes, over the decode (each window's steps incl. its <|endoftext|>)
                   "active_row_fraction": (round(sum(n + 1 for n in pipe.last.get("all_tokens", toks))
                                                 / pipe.last["gen_stats"]["row_steps"], 4)
                                           if pipe.last["gen_stats"].get("row_steps") else None),
                   "corpus": args.workload,
                   "token_crc32": pipe.last["crc"],
                   "parallelism": f"window-shard x{world}",
                   "weights": (f"synthetic seed 0, random-init + planted eot_after={args.eot_after}" if args.random_weights
                               else f"synthetic seed 0, random-init + margin-planted decoder program (weights.py plant {plant})")},
        "stages_s_per_step": {k: round(v / args.steps, 4) for k, v in stage_timed.items()},
    }
    if world > 1:
        out["ranks"] = [{"elapsed_s": round(r[0], 3), "windows": int(r[1]), "tokens": int(r[2]), "decoder_steps": int(r[3])}
                        for r in rank_info]
        out["config"]["shard_balance"] = args.balance
    if os.environ.get("VLOG_AMD_BENCH_SHARE_GPU") == "1":
        # a rehearsal of the N > 1 path with several ranks on one device: NOT a scaling result
        out["config"]["gpus_shared"] = True
        out["config"]["physical_gpus"] = torch.cuda.device_count()
    if prof:
        out.update(roofline_block(breakdown, prof, dom, args, beam=args.beam))
    comp = composite_roofline(dims, toks, pipe.last["steps"], len(pipe.prompt), elapsed / args.steps, W)
    out.setdefault("roofline", {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                                "traffic": None})
    out["roofline"]["composite"] = comp
    if parity is not None:
        out["parity"] = parity
    if world == 1 and not args.no_cpu_baseline and sd is not None:
        try:
            out["cpu_baseline"] = cpu_baseline(dims, sd, mean_tok)
        except Exception as e:  # reported, never fatal to the GPU measurement
            out["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
    if run_var:
        del pipe, eng, pcm_dev, sd
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        vsteps = args.variable_steps or max(2, args.steps // 4)
        try:
            out["variable"] = variable_block(args, dims, base_sd, tok, local, vsteps)
        except Exception as e:  # reported, never fatal to the headline measurement
            out["variable"] = {"error": str(e)[:300]}
    if json_fd is not None:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    else:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
