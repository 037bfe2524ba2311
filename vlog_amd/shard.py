"""Window sharding over the GPUs of one node: one process per GPU, no data-path collective.

A long file's 30 s windows are partitioned into contiguous ranges, one per GPU.  Each shard computes the log-mel
frames of its own range from its PCM slice (plus 200-sample margins: the STFT frames straddle the boundary, and
the reflect padding only applies at the file edges, so shard frames equal the whole-file frames bit for bit).
The single cross-shard value is the faster-whisper GLOBAL log-mel max (max(x, gmax - 8) over the whole file): each
shard reports its local max, the coordinator takes the max, every shard clamps with it.  Shards then encode and
decode their windows independently and return segments, which the coordinator merges in time order.

Two launchers share the partition / exchange / merge logic:
  * `transcribe_sharded(...)`  — a coordinator process that never touches the GPU spawns one worker per GPU
    (multiprocessing "spawn") and talks to them over pipes;
  * `run_rank(...)`             — for torch.distributed-launched ranks (bench.py): the max is a one-float
    all_reduce(MAX) and the segments are gathered with gather_object.
"""
from __future__ import annotations

import multiprocessing as mp
import os
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .dims import HOP_LENGTH, N_FRAMES, N_FFT, SAMPLE_RATE

MARGIN = N_FFT // 2       # samples each side of a shard's range


def content_frames(n_samples: int) -> int:
    """faster-whisper: features.shape[-1] - 1 = (N + 160) // 160 - 1."""
    return (n_samples + HOP_LENGTH) // HOP_LENGTH - 1


def partition_windows(n_windows: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous, balanced [start, end) window ranges (the first n % world shards get one more)."""
    q, r = divmod(n_windows, world)
    out, s = [], 0
    for i in range(world):
        e = s + q + (1 if i < r else 0)
        out.append((s, e))
        s = e
    return out


# ----------------------------------------------------------------------------------- expected work per window
# A window's decode cost follows its token count (the decoder steps), which follows how much of it is speech.
# The estimate below is the scheduler's only view of it: speech seconds from the per-frame log energy the VAD
# stand-in already computes on the GPU (wm_frame_energy), within 40 dB of the file's loud frames, times a
# speaking rate.  Only its order and relative size matter: the row-set decode starts the longest-expected
# windows first (so the short ones fill in behind them: longest-processing-time-first), and the shard partition
# balances the expected tokens per GPU instead of the window count.
TOKENS_PER_SPEECH_SECOND = 4.0


def speech_frames(frame_db: np.ndarray) -> np.ndarray:
    """Frames within 40 dB of the file's loud frames (its 99th-percentile frame) and above -70 dBFS."""
    db = np.asarray(frame_db, dtype=np.float64)
    finite = db[db > -100.0]
    peak = float(np.percentile(finite, 99)) if finite.size else -100.0
    return db > max(peak - 40.0, -70.0)


def expected_tokens(frame_db: np.ndarray, frame: int, starts: Sequence[int], lengths: Sequence[int]) -> np.ndarray:
    """Expected tokens of each window [starts[i], starts[i] + lengths[i]) (samples) from per-frame dB of `frame`
    samples: speech seconds x TOKENS_PER_SPEECH_SECOND, at least 1."""
    sp = speech_frames(frame_db).astype(np.int64)
    csum = np.concatenate([[0], np.cumsum(sp)])
    out = np.empty(len(starts), dtype=np.float64)
    for i, (s, n) in enumerate(zip(starts, lengths)):
        a = min(len(sp), s // frame)
        b = min(len(sp), max(a, -(-(s + n) // frame)))
        out[i] = max(1.0, (csum[b] - csum[a]) * frame / SAMPLE_RATE * TOKENS_PER_SPEECH_SECOND)
    return out


def expected_token_order(tokens: Sequence[float]) -> List[int]:
    """Window indices longest-expected first (stable)."""
    return [int(i) for i in np.argsort(-np.asarray(tokens, dtype=np.float64), kind="stable")]


def partition_by_weight(weights: Sequence[float], world: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) window ranges, one per rank, with the summed weights (expected tokens) as equal as
    contiguity allows: rank r ends where the running sum first reaches (r + 1) / world of the total, at the nearer
    window boundary; every rank keeps at least one window while windows remain."""
    w = np.asarray(weights, dtype=np.float64)
    n = w.size
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    csum = np.concatenate([[0.0], np.cumsum(w)])
    total = csum[-1]
    out, s = [], 0
    for r in range(world):
        if r == world - 1:
            e = n
        else:
            target = total * (r + 1) / world
            e = int(np.searchsorted(csum, target))              # csum[e] >= target
            if e > 0 and target - csum[e - 1] < csum[min(e, n)] - target:
                e -= 1
            e = max(e, s + 1 if s < n else s)                   # at least one window
            e = min(e, n - max(0, min(world - 1 - r, n - s - 1)))   # and one for each later rank, while they last
        out.append((s, e))
        s = e
    return out


@dataclass
class ShardPlan:
    rank: int
    win0: int
    win1: int
    frame0: int
    n_frames: int              # frames this shard computes ([frame0, frame0 + n_frames) of the file)
    sample0: int               # first PCM sample the shard receives
    sample1: int
    windows: List[Tuple[int, int]]   # (seek relative to frame0, size) per window
    offsets: List[float]             # absolute window start times (s)


def plan_shards(n_samples: int, world: int, weights: Optional[Sequence[float]] = None) -> List[ShardPlan]:
    """Per-rank plans; `weights` (expected tokens per window, expected_tokens) balances the work instead of the
    window count."""
    cf = content_frames(n_samples)
    n_win = max(1, -(-cf // N_FRAMES))
    plans = []
    parts = partition_by_weight(weights, world) if weights is not None else partition_windows(n_win, world)
    if weights is not None and len(weights) != n_win:
        raise ValueError(f"plan_shards: {len(weights)} weights for {n_win} windows")
    for rank, (w0, w1) in enumerate(parts):
        f0 = min(w0 * N_FRAMES, (cf + 1) & ~1)   # even: the log-mel kernel transforms (even, odd) frame pairs
        f1 = min(cf, w1 * N_FRAMES)
        if w1 == n_win and w1 > w0:
            f1 = cf + 1                      # the shard with the last window also owns the trailing frame
        nf = max(0, f1 - f0)
        s0 = max(0, f0 * HOP_LENGTH - MARGIN)
        s1 = min(n_samples, f1 * HOP_LENGTH + MARGIN)
        wins = [((w - w0) * N_FRAMES, min(N_FRAMES, cf - w * N_FRAMES)) for w in range(w0, w1)]
        plans.append(ShardPlan(rank, w0, w1, f0, nf, s0, s1, wins, [w * N_FRAMES * HOP_LENGTH / SAMPLE_RATE for w in range(w0, w1)]))
    return plans


def merge_segments(parts: Sequence[Sequence[dict]]) -> List[dict]:
    segs = [s for p in parts for s in p]
    segs.sort(key=lambda s: (s["start"], s["end"]))
    return segs


# ----------------------------------------------------------------------------------- per-shard work
def shard_features(engine, pcm_slice: np.ndarray, plan: ShardPlan, n_samples: int):
    import torch
    if plan.n_frames == 0:                   # more GPUs than windows: nothing to contribute
        return None, None, float("-inf")
    mel, gmax = engine.logmel(torch.from_numpy(np.ascontiguousarray(pcm_slice, dtype=np.float32)), n_samples=n_samples,
                              pcm_offset=plan.sample0, frame0=plan.frame0, n_frames=max(plan.n_frames, 1))
    return mel, gmax, engine.gmax_value(gmax)


def shard_decode(pipeline, mel, gmax, gmax_value: float, plan: ShardPlan, tokenizer, options) -> List[dict]:
    if not plan.windows:
        return []
    pipeline.model.engine.logmel_finalize(mel, gmax, gmax_value)
    results = pipeline.decode_windows(mel, plan.windows, plan.offsets, tokenizer, options, seed=plan.win0)
    out = []
    for wr in results:
        wr.seek += plan.frame0            # absolute seek for the segment records
        for s in pipeline.window_segments(wr, tokenizer, options):
            text = tokenizer.decode(s["tokens"])
            if s["start"] == s["end"] or not text.strip():
                continue
            out.append(dict(start=s["start"], end=s["end"], text=text, tokens=list(s["tokens"]),
                            avg_logprob=wr.avg_logprob, no_speech_prob=wr.no_speech_prob, temperature=wr.temperature))
    return out


# ----------------------------------------------------------------------------------- torch.distributed ranks
def run_rank(pipeline, pcm: np.ndarray, n_samples: int, tokenizer, options, rank: int, world: int,
             group=None, gather: bool = True) -> Optional[List[dict]]:
    """Rank `rank` of `world` (torch.distributed already initialised): returns merged segments on rank 0."""
    import torch
    import torch.distributed as dist
    plan = plan_shards(n_samples, world)[rank]
    mel, gmax, local = shard_features(pipeline.model.engine, pcm[plan.sample0: plan.sample1], plan, n_samples)
    t = torch.tensor([local], dtype=torch.float32)
    if dist.get_backend(group) == "nccl":
        t = t.to(pipeline.model.engine.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    segs = shard_decode(pipeline, mel, gmax, float(t.item()), plan, tokenizer, options)
    if not gather:
        return segs
    parts = [None] * world if rank == 0 else None
    dist.gather_object(segs, parts, dst=0, group=group)
    return merge_segments(parts) if rank == 0 else None


# ----------------------------------------------------------------------------------- spawn-based coordinator
def _worker(conn, device: int, model_spec: str, model_kwargs: dict):
    os.environ["VLOG_AMD_DEVICE"] = str(device)
    from .transcribe import BatchedInferencePipeline, WhisperModel
    model = WhisperModel(model_spec, device="cuda", device_index=device, **model_kwargs)
    pipe = BatchedInferencePipeline(model)
    state: Dict[str, Any] = {}
    conn.send(("ready", device))
    while True:
        msg = conn.recv()
        kind = msg[0]
        try:
            if kind == "features":
                _, pcm_slice, plan, n_samples = msg
                mel, gmax, local = shard_features(model.engine, pcm_slice, plan, n_samples)
                state.update(mel=mel, gmax=gmax, plan=plan)
                conn.send(("max", local))
            elif kind == "decode":
                _, gmax_value, language, task, opt_kwargs = msg
                from .transcribe import TranscriptionOptions
                tok = model.tokenizer(task=task, language=language)
                opts = TranscriptionOptions(**opt_kwargs)
                opts.suppress_tokens = list(tok.suppressed_tokens(opt_kwargs.get("suppress_tokens") or [-1]))
                segs = shard_decode(pipe, state["mel"], state["gmax"], gmax_value, state["plan"], tok, opts)
                state.clear()
                conn.send(("segments", segs))
            elif kind == "stop":
                conn.send(("stopped", device))
                return
        except Exception as e:          # reported to the coordinator, which raises
            conn.send(("error", f"{type(e).__name__}: {e}"))


class ShardedTranscriber:
    """Coordinator for N GPU worker processes.  Construct it before this process touches the GPU."""

    def __init__(self, model_spec: str, devices: Sequence[int], **model_kwargs):
        try:
            import torch
            if torch.cuda.is_initialized():
                raise RuntimeError("ShardedTranscriber must be created before the coordinator process uses the GPU")
        except ImportError:
            pass
        ctx = mp.get_context("spawn")
        self.conns, self.procs = [], []
        for d in devices:
            a, b = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(b, d, model_spec, model_kwargs), daemon=True)
            p.start()
            self.conns.append(a)
            self.procs.append(p)
        for c in self.conns:
            self._expect(c, "ready")

    @staticmethod
    def _expect(conn, kind):
        msg = conn.recv()
        if msg[0] == "error":
            raise RuntimeError(msg[1])
        if msg[0] != kind:
            raise RuntimeError(f"unexpected worker reply {msg[0]!r}")
        return msg[1]

    def transcribe(self, audio: np.ndarray, language: str = "en", task: str = "transcribe", **opt_kwargs) -> List[dict]:
        from .transcribe import default_batched_options
        n = audio.shape[0]
        world = len(self.conns)
        plans = plan_shards(n, world)
        for c, p in zip(self.conns, plans):
            c.send(("features", audio[p.sample0: p.sample1], p, n))
        gmax = max(self._expect(c, "max") for c in self.conns)
        okw = default_batched_options(**opt_kwargs)
        for c in self.conns:
            c.send(("decode", gmax, language, task, okw))
        return merge_segments([self._expect(c, "segments") for c in self.conns])

    def close(self):
        for c in self.conns:
            try:
                c.send(("stop",))
            except Exception:
                pass
        for p in self.procs:
            p.join(timeout=30)
