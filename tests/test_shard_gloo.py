"""Window sharding across ranks (vlog_amd/shard.py) on CPU with torch.distributed gloo, world size 1 vs 2.

The GPU engine is replaced by a test-only numpy stand-in that computes a shard's log-mel frames from ITS PCM
SLICE ONLY (samples outside the slice are NaN), so a plan with missing STFT margins fails; "decoding" turns
each window's features into deterministic pseudo-tokens.  Checks: shard frames equal the whole-file frames,
the global-max exchange, and that world 2's merged segments equal world 1's.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from oracle import mel as omel
from vlog_amd import shard
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.segments import split_segments_by_timestamps
from vlog_amd.tokenizer import Tokenizer

N_MELS = 80


class FakeEngine:
    device = "cpu"

    def logmel(self, pcm, n_samples, pcm_offset, frame0, n_frames):
        x = np.full(n_samples, np.nan)
        x[pcm_offset: pcm_offset + pcm.numel()] = pcm.numpy()
        raw = omel.log_mel_unclamped(np.nan_to_num(x, nan=1e6), N_MELS)     # poison: NaN -> huge
        full = omel.log_mel_unclamped(np.nan_to_num(x, nan=-1e6), N_MELS)
        seg = raw[:, frame0: frame0 + n_frames]
        assert np.array_equal(seg, full[:, frame0: frame0 + n_frames]), "shard used samples outside its slice"
        return torch.from_numpy(seg.astype(np.float32)), None

    def gmax_value(self, gmax_unused, _cache={}):
        raise AssertionError("not used")

    def logmel_finalize(self, mel, gmax, value):
        mel.copy_(torch.from_numpy(omel.clamp_and_scale(mel.numpy().astype(np.float64), value).astype(np.float32)))


class FakeModel:
    def __init__(self):
        self.engine = FakeEngine()


class WR:
    def __init__(self, seek, size, off, tokens):
        self.seek, self.size, self.time_offset, self.tokens = seek, size, off, tokens
        self.avg_logprob, self.no_speech_prob, self.temperature, self.compression_ratio = -0.3, 0.01, 0.0, 1.2


class FakePipeline:
    def __init__(self):
        self.model = FakeModel()

    def decode_windows(self, mel, windows, offsets, tok, options, seed=0):
        out = []
        tb = tok.timestamp_begin
        for (s, n), off in zip(windows, offsets):
            w = mel[:, s: s + n].numpy()
            h = int(abs(float(w.sum())) * 1000) % 997
            toks = [tb, 300 + h, 301 + (h * 7) % 500, tb + min(n // 2, 1500), tb + min(n // 2, 1500), 400 + h, tb + n // 2]
            out.append(WR(s, n, off, toks))
        return out

    def window_segments(self, wr, tok, options):
        segs, _, _ = split_segments_by_timestamps(wr.tokens, tok.timestamp_begin, wr.time_offset, wr.size,
                                                  wr.size * 0.01, wr.seek)
        return segs


def _global_max(x):
    return float(omel.log_mel_unclamped(x, N_MELS).max())


def _run(rank, world, port, x, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tok = Tokenizer(model_dims("tiny"), language="en")
    orig = shard.shard_features

    def feats(engine, pcm_slice, plan, n_samples):
        mel, _ = engine.logmel(torch.from_numpy(pcm_slice), n_samples, plan.sample0, plan.frame0, max(plan.n_frames, 1))
        return mel, None, float(mel.max())

    shard.shard_features = feats
    try:
        segs = shard.run_rank(FakePipeline(), x, x.size, tok, None, rank, world)
    finally:
        shard.shard_features = orig
    if rank == 0:
        q.put(segs)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, x):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run, args=(r, world, port, x, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_plan_covers_file_exactly():
    for n in [16000, 480000, 480160, 16000 * 95 + 7, 16000 * 3600]:
        for world in [1, 2, 3, 8]:
            plans = shard.plan_shards(n, world)
            frames = sum(p.n_frames for p in plans)
            assert frames == shard.content_frames(n) + 1
            wins = [w for p in plans for w in p.windows]
            assert sum(s for _, s in wins) == shard.content_frames(n)


def test_sharded_equals_single_gloo():
    x = np.concatenate([speech_like(30.0, 500 + i) for i in range(3)] + [speech_like(11.0, 503)])
    one = _launch(1, x)
    two = _launch(2, x)
    assert len(one) == len(two) > 0
    for a, b in zip(one, two):
        assert a["tokens"] == b["tokens"] and a["start"] == b["start"] and a["end"] == b["end"]
