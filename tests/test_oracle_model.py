"""oracle/model.py pinned against transformers WhisperForConditionalGeneration on identical seeded weights."""
import numpy as np
import torch
from transformers import WhisperConfig, WhisperForConditionalGeneration

from oracle.model import OracleWhisper
from vlog_amd.dims import custom_dims
from vlog_amd.weights import synthetic_state_dict


def _pair(n_mels=80):
    dims = custom_dims("t", n_mels, 128, 2, 2, 2, 51865, True)
    sd = synthetic_state_dict(dims, 1)
    cfg = WhisperConfig(vocab_size=51865, num_mel_bins=n_mels, encoder_layers=2, decoder_layers=2,
                        encoder_attention_heads=2, decoder_attention_heads=2, d_model=128, encoder_ffn_dim=512,
                        decoder_ffn_dim=512, max_source_positions=1500, max_target_positions=448)
    hf = WhisperForConditionalGeneration(cfg).eval()
    missing, unexpected = hf.load_state_dict(sd, strict=False)
    assert not unexpected and set(missing) <= {"proj_out.weight"}
    return dims, hf, OracleWhisper({k: v.numpy() for k, v in sd.items()}, dims, np.float64)


def test_encoder_and_decoder_match_transformers():
    dims, hf, orc = _pair(128)
    mel = np.random.default_rng(0).standard_normal((1, 128, 3000)).astype(np.float32)
    with torch.no_grad():
        enc_hf = hf.model.encoder(torch.from_numpy(mel)).last_hidden_state.numpy()
    enc = orc.encode(mel)
    assert np.abs(enc - enc_hf).max() < 1e-4
    st = dims.specials
    toks = np.array([[st.sot, st.lang_token("en"), st.transcribe, st.timestamp_begin, 400, 1234]])
    with torch.no_grad():
        lg_hf = hf(encoder_outputs=(torch.from_numpy(enc_hf),), decoder_input_ids=torch.from_numpy(toks)).logits.numpy()
    cross = orc.cross_kv(enc)
    a, cache = orc.decode(toks[:, :3], cross)
    b, _ = orc.decode(toks[:, 3:], cross, cache, offset=3)        # KV-cached continuation
    assert np.abs(np.concatenate([a, b], 1) - lg_hf).max() < 1e-4


def test_bf16_format_modes_stay_within_rounding_noise():
    """The engine-numeric-format modes (bf16_enc encoder, bf16_acts decoder) differ from the float32 restatement
    only by bf16 rounding; the teacher-forced parity helper finds an oracle-generated sequence identical to
    itself (tests/parity_util.py)."""
    from oracle.decode import GenerateOptions, generate_one
    from tests.parity_util import teacher_force
    from vlog_amd.weights import round_bf16
    dims = custom_dims("t", 80, 128, 2, 2, 2, 51865, True)
    sd = round_bf16(synthetic_state_dict(dims, 2, eot_after=20))
    mel = np.random.default_rng(1).standard_normal((1, 80, 3000)).astype(np.float32)
    f32 = OracleWhisper(sd, dims, np.float32)
    bf = OracleWhisper(sd, dims, np.float32, bf16_acts=True, bf16_enc=True)
    e32, ebf = f32.encode(mel), bf.encode(mel)
    rms = float(np.sqrt(np.mean(e32 ** 2)))
    assert np.abs(e32 - ebf).max() < 0.05 * rms and np.abs(e32 - ebf).mean() < 0.01 * rms
    st = dims.specials
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    opt = GenerateOptions(suppress_tokens=[st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm], max_length=60)
    cross = bf.cross_kv(ebf)
    r = generate_one(bf, cross, prompt, st, opt)
    chosen, best, score, ns = teacher_force(bf, cross, prompt, r.tokens, st, opt, len(prompt) + len(r.tokens) < 60)
    assert np.all(chosen - best >= -1e-9) and abs(score - r.score) < 1e-6 and abs(ns - r.no_speech_prob) < 1e-9


def test_bf16_rounding_forms_bit_identical():
    """oracle.model.to_bf16 (PyTorch's float32 -> bfloat16 conversion, used for speed) equals the integer
    round-to-nearest-even definition to_bf16_bits bit for bit, ties, subnormals, overflow and non-finite
    values included."""
    from oracle.model import to_bf16, to_bf16_bits
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(200000) * np.exp(rng.uniform(-90, 90, 200000))).astype(np.float32)
    ties = (rng.integers(0, 1 << 31, 4096, dtype=np.uint32) & np.uint32(0xFFFF0000)) | np.uint32(0x8000)
    edge = np.array([np.inf, -np.inf, np.nan, 0.0, -0.0, 3.4e38, -3.4e38, 3.3895e38, 1e-45, -1e-45, 1e-40],
                    dtype=np.float32)
    x = np.concatenate([x, ties.view(np.float32), edge])
    a, b = to_bf16(x), to_bf16_bits(x)
    fin = ~np.isnan(x)
    assert np.array_equal(a.view(np.uint32)[fin], b.view(np.uint32)[fin])
    assert np.isnan(a[~fin]).all()
