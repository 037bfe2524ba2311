"""Encoder self-attention kernel (wm_encoder_attention, the kernel wm_encode runs per layer) vs a float32
PyTorch reference of the same op on identical bf16 inputs, T = 1500 (the last 64-key tile is ragged).

Cases follow cdna_hip_programming.md §5.4 rule 26 for the online softmax's deferred rescale: besides plain
random data, inputs that FORCE the rescale branch mid-stream (a key whose score jumps far above everything
seen before, placed in a late tile) and the opposite (the row maximum in the very first tile).
Tolerance: bf16 output of an fp32-accumulated kernel whose P is rounded to bf16 (values up to 2^8 under the
deferred rescale): max abs error <= 2e-2 relative to max |O|, mean <= 2e-3."""
import pytest
import torch

from vlog_amd.dims import model_dims
from vlog_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

T = 1500


@pytest.fixture(scope="module")
def eng():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    return GpuEngine(dims, synthetic_state_dict(dims, seed=1, eot_after=40), 0)


def _reference(qkv: torch.Tensor, H: int) -> torch.Tensor:
    B, T_, three_d = qkv.shape
    d = three_d // 3
    x = qkv.float().view(B, T_, 3, H, 64).permute(2, 0, 3, 1, 4)       # [3][B][H][T][64]
    q, k, v = x[0], x[1], x[2]
    s = (q @ k.transpose(-1, -2)) * 0.125
    o = torch.softmax(s, dim=-1) @ v                                    # [B][H][T][64]
    return o.permute(0, 2, 1, 3).reshape(B, T_, d)


def _check(eng, qkv):
    got = eng.encoder_attention(qkv).float()
    ref = _reference(qkv, eng.dims.n_head)
    err = (got - ref).abs()
    scale = ref.abs().max().item()
    assert err.max().item() <= 2e-2 * scale, (err.max().item(), scale)
    assert err.mean().item() <= 2e-3 * scale, (err.mean().item(), scale)


@pytest.mark.parametrize("seed,amp", [(0, 1.0), (1, 3.0)])
def test_attention_random(eng, seed, amp):
    d = eng.dims.n_state
    g = torch.Generator().manual_seed(seed)
    qkv = (torch.randn(2, T, 3 * d, generator=g) * amp).to(torch.bfloat16).cuda()
    _check(eng, qkv)


def test_attention_forced_rescale(eng):
    """Scores stay small for 20 tiles, then one key per head jumps ~32 above: the deferred rescale must fire
    mid-stream and rescale O and l exactly once."""
    d, H = eng.dims.n_state, eng.dims.n_head
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, T, 3, H, 64, generator=g) * 0.5
    x[0, :, 0] = 1.0                                                  # every query = (1, ..., 1)
    x[0, 1300, 1] = 4.0                                               # key 1300: score 4*64/8 = 32 vs ~0
    x[0, 37, 1] = -4.0                                                # a very negative key in tile 0
    qkv = x.reshape(1, T, 3 * d).to(torch.bfloat16).cuda()
    _check(eng, qkv)


def test_attention_max_in_first_tile(eng):
    d, H = eng.dims.n_state, eng.dims.n_head
    g = torch.Generator().manual_seed(6)
    x = torch.randn(1, T, 3, H, 64, generator=g) * 0.5
    x[0, :, 0] = 1.0
    x[0, 3, 1] = 3.0                                                  # the row maximum sits in tile 0
    x[0, 1499, 1] = 2.5                                               # runner-up in the ragged last tile
    qkv = x.reshape(1, T, 3 * d).to(torch.bfloat16).cuda()
    _check(eng, qkv)
