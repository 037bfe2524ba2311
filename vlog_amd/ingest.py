"""Streaming ingest: s16le PCM from a pipe straight into device memory, log-mel computed
while the audio is still arriving.

The reference worker extracts audio with ffmpeg into a temporary WAV file and faster-whisper then reads and
decodes that file (reference worker/transcription.py:259-299, 342-351).  Here the bytes of
`ffmpeg ... -f s16le -ac 1 -ar 16000 -` (or any producer of 16 kHz mono s16le) are read from the pipe into
pinned host staging buffers, copied to the device asynchronously (double-buffered: the next read overlaps the
previous copy), converted on the device (`wm_pcm_from_s16`), and every log-mel frame whose 400-sample window
lies inside the samples received so far is computed right away (`wm_logmel` on that frame range).  At EOF the
remaining frames (those touching the end padding) are computed with the true length and the whole matrix is
normalised with the file's global max (`wm_logmel_finalize`), exactly as the one-shot path does — so the
features are bit-identical to `engine.features(pcm)` (tests/test_gpu_ingest.py).
"""
from __future__ import annotations

import ctypes as C
import shutil
import subprocess
from dataclasses import dataclass
from typing import BinaryIO, List, Optional

import numpy as np
import torch

from . import _capi
from .audio import SR as SAMPLE_RATE

HOP_LENGTH = 160

N_FFT = 400


@dataclass
class IngestResult:
    pcm: torch.Tensor          # f32 [n] on the device
    features: torch.Tensor     # finalised log-mel [n_mels, n // 160 + 1] on the device
    n_samples: int

    @property
    def duration(self) -> float:
        return self.n_samples / SAMPLE_RATE


class StreamingIngest:
    def __init__(self, engine, staging_samples: int = 1 << 20, initial_capacity: int = SAMPLE_RATE * 600):
        self.eng = engine
        self.dev = engine.device
        self.stage = [torch.empty(staging_samples, dtype=torch.int16, pin_memory=True) for _ in range(2)]
        self.stage_ev: List[Optional[torch.cuda.Event]] = [None, None]
        self.stage_dev = torch.empty(staging_samples, dtype=torch.int16, device=self.dev)
        self.pcm = torch.empty(max(initial_capacity, 1), dtype=torch.float32, device=self.dev)
        self.n = 0                       # samples received
        self.done = 0                    # log-mel frames computed
        self.mels: List[torch.Tensor] = []
        self.gmax = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._carry = b""                # an odd trailing byte between reads
        self._k = 0

    # -- device PCM
    def _reserve(self, n: int) -> None:
        if n <= self.pcm.numel():
            return
        cap = self.pcm.numel()
        while cap < n:
            cap *= 2
        grown = torch.empty(cap, dtype=torch.float32, device=self.dev)
        grown[: self.n].copy_(self.pcm[: self.n])
        self.pcm = grown

    def feed(self, data) -> None:
        """Append s16le bytes (or an int16 array)."""
        if isinstance(data, np.ndarray):
            samples = np.ascontiguousarray(data, dtype=np.int16)
        else:
            buf = self._carry + bytes(data)
            cut = len(buf) & ~1
            self._carry = buf[cut:]
            samples = np.frombuffer(buf[:cut], dtype=np.int16)
        cap = self.stage[0].numel()
        for o in range(0, samples.size, cap):
            self._push(samples[o: o + cap])
        self._frames(final=False)

    def _push(self, s: np.ndarray) -> None:
        k = self._k
        self._k ^= 1
        if self.stage_ev[k] is not None:
            self.stage_ev[k].synchronize()          # the copy out of this pinned buffer has finished
        m = s.size
        self.stage[k][:m].numpy()[:] = s
        self._reserve(self.n + m)
        st = torch.cuda.current_stream(self.dev)
        self.stage_dev[:m].copy_(self.stage[k][:m], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(st)
        self.stage_ev[k] = ev
        with torch.cuda.device(self.dev):
            _capi.check(self.eng.lib.wm_pcm_from_s16(self.eng.h, C.c_void_p(self.stage_dev.data_ptr()), m,
                                                     C.c_void_p(self.pcm.data_ptr() + 4 * self.n),
                                                     self.eng.stream_ptr()), "wm_pcm_from_s16")
        self.n += m

    def _frames(self, final: bool) -> None:
        if final:
            ready = (self.n + HOP_LENGTH) // HOP_LENGTH          # N // 160 + 1 frames in all
        else:
            # frame f reads samples [160 f - 200, 160 f + 200): complete once 160 f + 200 <= n; frames are
            # transformed in (even, odd) pairs, so a chunk ends on an even frame (bit-identical to one shot)
            ready = max(0, (self.n - N_FFT // 2) // HOP_LENGTH + 1) if self.n >= N_FFT // 2 else 0
            ready &= ~1
        if ready <= self.done:
            return
        nf = ready - self.done
        mel = torch.empty((self.eng.dims.n_mels, nf), device=self.dev, dtype=torch.float32)
        with torch.cuda.device(self.dev):
            _capi.check(self.eng.lib.wm_logmel(self.eng.h, C.c_void_p(self.pcm.data_ptr()), 0, self.n, self.done, nf,
                                               C.c_void_p(mel.data_ptr()), nf, C.c_void_p(self.gmax.data_ptr()),
                                               self.eng.stream_ptr()), "wm_logmel")
        self.mels.append(mel)
        self.done = ready

    def finish(self) -> IngestResult:
        if self._carry:
            raise ValueError("odd number of bytes in an s16le stream")
        self._frames(final=True)
        mel = torch.cat(self.mels, dim=1) if len(self.mels) > 1 else self.mels[0]
        self.eng.logmel_finalize(mel, self.gmax)
        return IngestResult(self.pcm[: self.n], mel, self.n)


def ingest_pipe(engine, stream: BinaryIO, read_bytes: int = 1 << 20) -> IngestResult:
    """Read s16le 16 kHz mono PCM from `stream` (a pipe or file object) until EOF."""
    ing = StreamingIngest(engine)
    while True:
        b = stream.read(read_bytes)
        if not b:
            break
        ing.feed(b)
    return ing.finish()


def ffmpeg_pcm_command(path: str) -> List[str]:
    """The extraction the worker runs, writing raw PCM to stdout instead of a temporary WAV."""
    return ["ffmpeg", "-nostdin", "-loglevel", "error", "-i", path, "-vn", "-ac", "1", "-ar", str(SAMPLE_RATE),
            "-f", "s16le", "-"]


def ingest_media(engine, path: str) -> IngestResult:
    """ffmpeg -> pipe -> device.  Raises if ffmpeg is not installed (it is not in this build image; the
    tests drive ingest_pipe with a simulated s16le producer)."""
    exe = shutil.which("ffmpeg")
    if exe is None:
        raise RuntimeError("ffmpeg not found")
    with subprocess.Popen(ffmpeg_pcm_command(path), stdout=subprocess.PIPE) as p:
        res = ingest_pipe(engine, p.stdout)
        if p.wait() != 0:
            raise RuntimeError(f"ffmpeg failed on {path}")
    return res
