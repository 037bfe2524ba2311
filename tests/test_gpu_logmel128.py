"""The log-mel front end at large-v3's 128 mel bins (the headline model; configs 4 and 5) vs oracle/mel.py.

north_star gate: log-mel max-abs <= 1e-4 (faster-whisper FeatureExtractor semantics, the global max - 8 clamp over
the whole file).  The 80-mel checks live in tests/test_gpu_parity.py; here the 128-row slaney
filterbank the engine builds at wm_create (vlog_amd/csrc/engine.cpp build_frontend) runs on the device for
1 s, 30 s, 61.3 s and a 1 h file (360,001 frames under ONE global clamp), plus the shard form the window-sharded
bench uses (each rank's frames from its PCM slice +-200 samples, the clamp from the host max of the shard maxima).
The engine is a front-end-only handle of model_dims("large-v3") (GpuEngine.frontend: no weights, same kernels);
the full large-v3 engine's features() on the bench's 150 windows is checked in tests/test_gpu_configs.py.
Reference call: worker/transcription.py:105-111 (model.transcribe on the WAV path).
"""
import numpy as np
import pytest
import torch

from oracle import mel as omel
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def eng():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("large-v3")
    assert dims.n_mels == 128
    return GpuEngine.frontend(dims, 0)


@pytest.mark.parametrize("seconds,seed", [(1.0, 31), (30.0, 32), (61.3, 33)])
def test_logmel128_matches_oracle(eng, seconds, seed):
    x = speech_like(seconds, seed)
    ref = omel.log_mel(x, 128)
    got = eng.features(torch.from_numpy(x)).cpu().numpy()
    assert got.shape == ref.shape == (128, x.size // 160 + 1)
    err = float(np.abs(got - ref).max())
    assert err <= TOL, err


def test_logmel128_one_hour_global_clamp(eng):
    """1 h = 120 concatenated 30 s clips: the clamp floor is the max over all 360,001 frames."""
    x = np.concatenate([speech_like(30.0, 600 + i) for i in range(120)])
    ref = omel.log_mel(x, 128)
    got = eng.features(torch.from_numpy(x)).cpu().numpy()
    assert got.shape == ref.shape == (128, 360001)
    err = np.abs(got - ref)
    assert float(err.max()) <= TOL, (float(err.max()), np.unravel_index(int(err.argmax()), err.shape))
    # the clamp is active (silence between syllables sits at the floor) and it is the whole file's
    assert np.isclose(ref.min(), ref.max() - 2.0, atol=1e-6)
    assert np.isclose(got.min(), ref.min(), atol=TOL)


def test_logmel128_shards_equal_whole_file(eng):
    """Shard frames from PCM slices (+-200 samples), the global max exchanged as one host float: bit-identical to the
    whole-file features, and within the gate of the oracle."""
    x = np.concatenate([speech_like(30.0, 700 + i) for i in range(6)]) [: 16000 * 171 + 37]
    N = x.size
    whole = eng.features(torch.from_numpy(x))
    nf = N // 160 + 1
    cuts = [0, 3000, 9000, 12000, nf]
    parts, maxima = [], []
    for f0, f1 in zip(cuts[:-1], cuts[1:]):
        s0, s1 = max(0, f0 * 160 - 200), min(N, f1 * 160 + 200)
        mel, gmax = eng.logmel(torch.from_numpy(x[s0:s1].copy()), n_samples=N, pcm_offset=s0, frame0=f0,
                               n_frames=f1 - f0)
        parts.append((mel, gmax))
        maxima.append(eng.gmax_value(gmax))
    g = max(maxima)
    for mel, gmax in parts:
        eng.logmel_finalize(mel, gmax, gmax_value=g)
    parts = [p for p, _ in parts]
    sharded = torch.cat(parts, dim=1)
    assert torch.equal(sharded, whole)
    ref = omel.log_mel(x, 128)
    assert float(np.abs(sharded.cpu().numpy() - ref).max()) <= TOL
