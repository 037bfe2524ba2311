"""CPU: the Silero VAD v5 restatement (oracle/vad_net.py) and the weight loader (vlog_amd/silero.py).

Silero's weights are not in this image, so the network's parity with Silero itself is unpinned;
these tests pin the pieces that do not depend on the weights: the window/context layout faster-whisper 1.1
feeds the encoder, the padding of get_speech_timestamps, the STFT (the conv basis against numpy's rfft), the
LSTM recurrence against torch.nn.LSTMCell, and the file loader's name/shape checks."""
import numpy as np
import pytest
import torch

from oracle import vad_net
from vlog_amd import silero


def test_padding_and_window_context():
    assert len(vad_net.pad_audio(np.zeros(1000))) == 1024
    assert len(vad_net.pad_audio(np.zeros(1024))) == 1536        # a whole extra window at len % 512 == 0
    assert len(vad_net.pad_audio(np.zeros(0))) == 512
    a = np.arange(1536, dtype=np.float32)
    x = vad_net.window_inputs(a)
    assert x.shape == (3, 576)
    assert np.all(x[0, :64] == 0) and np.array_equal(x[0, 64:], a[:512])
    assert np.array_equal(x[1, :64], a[448:512]) and np.array_equal(x[2, :64], a[960:1024])


def test_stft_basis_is_hann_rfft():
    rng = np.random.default_rng(0)
    frame = rng.standard_normal(256)
    basis = silero.stft_basis()[:, 0, :].astype(np.float64)
    spec = basis @ frame
    ref = np.fft.rfft(frame * (0.5 - 0.5 * np.cos(2 * np.pi * np.arange(256) / 256)))
    assert np.allclose(spec[:129], ref.real, atol=1e-4) and np.allclose(spec[129:], ref.imag, atol=1e-4)


def test_encoder_shapes_and_reflection():
    wt = silero.synthetic_weights(1)
    rng = np.random.default_rng(2)
    x = rng.standard_normal((5, 576)) * 0.1
    f = vad_net.encoder(x, wt)
    assert f.shape == (5, 128) and np.all(f >= 0)
    # the right reflection: frame 3 covers samples 384..639 of [x, x[574..511]]
    xr = np.concatenate([x, x[:, 574:510:-1]], axis=1)
    assert np.array_equal(xr[:, 576], x[:, 574]) and np.array_equal(xr[:, 639], x[:, 511])


def test_decoder_matches_torch_lstmcell():
    wt = silero.synthetic_weights(3)
    rng = np.random.default_rng(4)
    feats = np.abs(rng.standard_normal((40, 128)))
    ours = vad_net.decoder(feats, wt)
    cell = torch.nn.LSTMCell(128, 128).double()
    with torch.no_grad():
        cell.weight_ih.copy_(torch.from_numpy(wt["decoder.rnn.weight_ih"]).double())
        cell.weight_hh.copy_(torch.from_numpy(wt["decoder.rnn.weight_hh"]).double())
        cell.bias_ih.copy_(torch.from_numpy(wt["decoder.rnn.bias_ih"]).double())
        cell.bias_hh.copy_(torch.from_numpy(wt["decoder.rnn.bias_hh"]).double())
        h = torch.zeros(1, 128, dtype=torch.float64)
        c = torch.zeros(1, 128, dtype=torch.float64)
        hw = torch.from_numpy(wt["decoder.decoder.2.weight"]).double().reshape(-1)
        hb = float(wt["decoder.decoder.2.bias"][0])
        ref = []
        for t in range(len(feats)):
            h, c = cell(torch.from_numpy(feats[t: t + 1]), (h, c))
            ref.append(float(torch.sigmoid(torch.relu(h[0]) @ hw + hb)))
    assert np.allclose(ours, ref, atol=1e-12)


def test_synthetic_weights_deterministic_and_shaped():
    a, b = silero.synthetic_weights(5), silero.synthetic_weights(5)
    assert set(a) == set(silero.WEIGHT_SHAPES)
    for k, shape in silero.WEIGHT_SHAPES.items():
        assert a[k].shape == shape and a[k].dtype == np.float32 and np.array_equal(a[k], b[k])
    assert not np.array_equal(a["decoder.rnn.weight_hh"], silero.synthetic_weights(6)["decoder.rnn.weight_hh"])


@pytest.mark.parametrize("fmt", ["npz", "safetensors"])
def test_weight_file_loader(tmp_path, fmt):
    wt = silero.synthetic_weights(7)
    named = {silero.PREFIX + k: v for k, v in wt.items()}
    named["_model.unused.extra"] = np.zeros(3, np.float32)
    path = str(tmp_path / f"silero.{fmt}")
    if fmt == "npz":
        np.savez(path, **named)
    else:
        from safetensors.numpy import save_file
        save_file(named, path)
    got = silero.resolve_weights(path)
    assert set(got) == set(wt) and all(np.array_equal(got[k], wt[k]) for k in wt)
    bad = dict(named)
    bad["_model.decoder.rnn.weight_hh"] = np.zeros((128, 128), np.float32)
    np.savez(str(tmp_path / "bad.npz"), **bad)
    with pytest.raises(ValueError, match="shape"):
        silero.resolve_weights(str(tmp_path / "bad.npz"))
    del bad["_model.decoder.rnn.weight_hh"]
    np.savez(str(tmp_path / "missing.npz"), **bad)
    with pytest.raises(ValueError, match="missing"):
        silero.resolve_weights(str(tmp_path / "missing.npz"))
    with pytest.raises(FileNotFoundError):
        silero.resolve_weights(str(tmp_path / "nope.npz"))
