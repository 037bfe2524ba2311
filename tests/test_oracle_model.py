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
