"""HIP path vs the CPU oracle on identical seeded inputs (runs on an MI355X; calls through the C-ABI).

Tolerances (BASELINE.json north_star): log-mel max-abs <= 1e-4; greedy tokens identical on >= 99 % of windows
at the generate boundary (identical encoder output + prompt).  Encoder output and logits are bf16-compute
vs float32-oracle, checked relative to the tensor scale (written per test).
"""
import numpy as np
import pytest
import torch

from oracle import mel as omel
from oracle.decode import GenerateOptions, generate_one
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiny():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=3, eot_after=60)
    eng = GpuEngine(dims, sd, 0)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32)
    orc.bf = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)   # engine numeric format (decoder)
    return dims, eng, orc


def _audio(seconds, seed):
    return speech_like(seconds, seed)


@pytest.mark.parametrize("seconds,seed", [(1.0, 1), (30.0, 2), (61.3, 3), (0.05, 4)])
def test_logmel_matches_oracle(tiny, seconds, seed):
    dims, eng, _ = tiny
    x = _audio(seconds, seed)
    ref = omel.log_mel(x, dims.n_mels)
    got = eng.features(torch.from_numpy(x)).cpu().numpy()
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-4


def test_logmel_silence_and_clipping(tiny):
    dims, eng, _ = tiny
    x = np.zeros(16000 * 3, dtype=np.float32)
    x[16000:16100] = 0.999                                    # click inside silence
    x[30000:] = np.sign(np.sin(np.arange(18000) * 0.3)) * 1.0  # clipped square wave
    ref = omel.log_mel(x, dims.n_mels)
    got = eng.features(torch.from_numpy(x)).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-4


def test_logmel_shard_equals_whole_file(tiny):
    """A shard computing frames [f0, f1) from its PCM slice (+-200 samples) equals the whole-file frames."""
    dims, eng, _ = tiny
    x = _audio(95.0, 7)
    N = x.size
    whole, g_whole = eng.logmel(torch.from_numpy(x))
    for f0, f1 in [(0, 3000), (3000, 6000), (9000, N // 160 + 1)]:
        s0 = max(0, f0 * 160 - 200)
        s1 = min(N, f1 * 160 + 200)
        part, _ = eng.logmel(torch.from_numpy(x[s0:s1].copy()), n_samples=N, pcm_offset=s0, frame0=f0, n_frames=f1 - f0)
        assert torch.equal(part, whole[:, f0:f1])


def test_encoder_matches_oracle(tiny):
    dims, eng, orc = tiny
    x = _audio(45.0, 11)
    feats = omel.log_mel(x, dims.n_mels)
    mel = torch.from_numpy(feats).cuda()
    seeks, lens = [0, 3000], [3000, feats.shape[1] - 1 - 3000]
    enc = eng.encode(mel, seeks, lens).float().cpu().numpy()
    segs = np.stack([omel.pad_or_trim(feats[:, s: s + n]) for s, n in zip(seeks, lens)])
    ref = orc.encode(segs)
    err = np.abs(enc - ref)
    # bf16 activations through 4 layers: bounded relative to the output scale (LayerNorm'd, O(1))
    assert err.max() < 0.15, err.max()
    assert err.mean() < 0.01, err.mean()


def test_teacher_forced_logits_bf16_oracle(tiny):
    """Against the oracle in the engine's numeric format the logits agree to summation-order noise."""
    dims, eng, orc = tiny
    st = dims.specials
    feats = omel.log_mel(_audio(30.0, 22), dims.n_mels)
    enc = eng.encode(torch.from_numpy(feats).cuda(), [0], [3000])
    eng.reserve(4, 4)
    eng.cross_kv(enc, 1)
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe] + list(range(500, 540))])
    logits, _ = eng.forward([1], toks)
    ref, _ = orc.bf.decode(toks, orc.bf.cross_kv(enc.float().cpu().numpy()))
    assert np.abs(logits.cpu().numpy() - ref).max() < 0.02


def test_teacher_forced_logits(tiny):
    dims, eng, orc = tiny
    st = dims.specials
    x = _audio(30.0, 21)
    feats = omel.log_mel(x, dims.n_mels)
    mel = torch.from_numpy(feats).cuda()
    enc = eng.encode(mel, [0], [3000])
    eng.reserve(4, 4)
    eng.cross_kv(enc, 0)
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe, st.timestamp_begin, 400, 1234, 50, st.timestamp_begin + 20]])
    logits, _ = eng.forward([0], toks)
    ref, _ = orc.decode(toks, orc.cross_kv(enc.float().cpu().numpy()))
    got = logits.cpu().numpy()
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() < 0.02 * scale + 1e-3


EPS = 0.02   # nats: the bf16 numeric noise floor of a logit (measured: ~0.006 max abs)


def test_greedy_matches_oracle(tiny):
    """Generate boundary, same encoder output.  Every GPU token, teacher-forced through the oracle with the
    same rules, must be within EPS of the oracle's best log-prob at that step (exact identity is
    ill-conditioned at near-ties of a random model); most windows are identical outright."""
    from oracle.decode import score_sequence
    dims, eng, orc = tiny
    st = dims.specials
    W = 6
    x = np.concatenate([_audio(30.0, 100 + i) for i in range(W)])
    feats = omel.log_mel(x, dims.n_mels)
    mel = torch.from_numpy(feats).cuda()
    enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W)
    eng.reserve(W, W)
    eng.cross_kv(enc, 0)
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    sup = [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]
    opt = GenerateOptions(suppress_tokens=sup, max_length=120)
    res, steps = eng.generate(list(range(W)), [prompt] * W, suppress_tokens=sup, max_length=120)
    encf = enc.float().cpu().numpy()
    same = 0
    for w in range(W):
        cross = orc.cross_kv(encf[w: w + 1])
        r = generate_one(orc, cross, prompt, st, opt)
        same += r.tokens == res[w].tokens
        assert abs(r.no_speech_prob - res[w].no_speech_prob) < 1e-3
        ended = len(prompt) + len(res[w].tokens) < 120
        chosen, best, score = score_sequence(orc, cross, prompt, res[w].tokens, st, opt, ended)
        assert np.all(chosen >= best - EPS), np.min(chosen - best)
        assert abs(score - res[w].score) < 2e-2 * max(1.0, abs(score))
    assert same >= W - 1, f"{same}/{W} windows identical"
