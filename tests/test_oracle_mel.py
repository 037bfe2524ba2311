"""oracle/mel.py pinned against transformers' WhisperFeatureExtractor numpy path (in-container third-party
oracle, [TF] feature_extraction_whisper.py:105-133, audio_utils.py:638-809)."""
import numpy as np
import pytest
from transformers import WhisperFeatureExtractor
from transformers.audio_utils import mel_filter_bank

from oracle import mel as omel
from vlog_amd.audio import speech_like


@pytest.mark.parametrize("n_mels", [80, 128])
def test_filterbank_matches_transformers(n_mels):
    ref = mel_filter_bank(num_frequency_bins=201, num_mel_filters=n_mels, min_frequency=0.0, max_frequency=8000.0,
                          sampling_rate=16000, norm="slaney", mel_scale="slaney")
    got = omel.mel_filters(n_mels).T
    assert np.allclose(got, ref, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("n_mels,seed", [(80, 0), (128, 1)])
def test_log_mel_matches_transformers(n_mels, seed):
    x = speech_like(30.0, seed)          # exactly 30 s: transformers pads nothing, faster-whisper padding=0
    fe = WhisperFeatureExtractor(feature_size=n_mels)
    ref = fe._np_extract_fbank_features(x[None], "cpu")[0]
    got = omel.log_mel(x, n_mels, padding=0)
    assert got.shape == ref.shape == (n_mels, 3000)
    assert np.abs(got - ref).max() < 2e-5


def test_frame_count_and_global_clamp():
    x = speech_like(61.3, 2)
    m = omel.log_mel(x, 80)
    assert m.shape[1] == (x.size + 160) // 160
    raw = omel.log_mel_unclamped(x, 80)
    assert np.isclose((m.min() * 4 - 4), raw.max() - 8, atol=1e-4)   # the global (whole-file) clamp
    assert np.allclose(omel.pad_or_trim(m[:, :100]), np.pad(m[:, :100], ((0, 0), (0, 2900))))
