"""The persistent encoder GEMM (one block per CU walking its tiles, the next tile's first K-tiles loaded during the
current tile's last K-steps and epilogue; gemm_8p.hip gemm_8pp_kernel) changes only the schedule: the encoder
output must be bit-identical to the one-block-per-tile kernel.  60 tiny windows put every encoder projection
(qkv, out, fc1, fc2: >= 512 tiles each) on the persistent path.  Runs through the C-ABI on the MI355X."""
import numpy as np
import pytest
import torch

from oracle import mel as omel
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

W = 60


def test_persistent_encoder_gemm_bit_identical():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=5, eot_after=40), 0)
    x = np.concatenate([speech_like(30.0, 900 + i) for i in range(W)])
    feats = torch.from_numpy(omel.log_mel(x, dims.n_mels)).cuda()
    seek, n = [3000 * i for i in range(W)], [3000] * W
    try:
        eng.set_option("gemm_persistent", 0)
        ref = eng.encode(feats, seek, n).clone()
        eng.set_option("gemm_persistent", 1)
        got = eng.encode(feats, seek, n)
    finally:
        eng.set_option("gemm_persistent", 0)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and torch.isfinite(got.float()).all()
    assert torch.equal(got, ref)
