"""The margin-planted synthetic model (vlog_amd/weights.py plant_margin) on the CPU oracle: the planted program
runs (the decoded tokens follow the script, branch tokens chosen by window-level audio bits, every segment
boundary a timestamp pair), the model is decisive (every step's top-1 / top-2 gap far above bf16 noise), its
output depends on the audio, and the gate checker (tests/parity_util.py gate_windows) passes between the
oracle's f32 and bf16-activation forms.  The GPU-side gates are tests/test_gpu_gates.py."""
import numpy as np
import pytest

from oracle import mel as omel
from oracle.decode import GenerateOptions, generate_one
from oracle.model import OracleWhisper
from tests.parity_util import assert_gates, gate_windows
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import margin_plan, round_bf16, synthetic_state_dict

W = 4


@pytest.fixture(scope="module")
def tiny():
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=0, plant="margin")
    w = round_bf16(sd)
    o32 = OracleWhisper(w, dims, np.float32)
    o16 = OracleWhisper(w, dims, np.float32, bf16_acts=True)
    # windows 1, 3, 6, 9 of the corpus: their bits differ (measured), so the test sees the audio dependence
    seeds = [1, 3, 6, 9]
    x = np.concatenate([speech_like(30.0, s) for s in seeds])
    mel = omel.log_mel(x, dims.n_mels)[:, :3000 * W].reshape(dims.n_mels, W, 3000).transpose(1, 0, 2)
    enc = o32.encode(np.ascontiguousarray(mel))
    tok = Tokenizer(dims, language="en")
    prompt = list(tok.sot_sequence)
    opt = GenerateOptions(suppress_tokens=list(tok.suppressed_tokens([-1])), max_length=448)
    res = [generate_one(o32, o32.cross_kv(enc[i:i + 1]), prompt, dims.specials, opt) for i in range(W)]
    return dims, o16, enc, tok, prompt, opt, res


def test_plan_followed_and_audio_dependent(tiny):
    dims, _, _, _, _, _, res = tiny
    plan = margin_plan(dims, 0)
    st = dims.specials
    choices = []
    for r in res:
        # every planted slot in order, exactly one token of each branch pair, timestamps doubled at boundaries
        flat = [t for t in r.tokens]
        k, pick = 0, []
        for slot, kind in zip(plan.slots, plan.kinds):
            assert flat[k] in slot, (k, flat[k], slot)
            if len(slot) == 2:
                pick.append(slot.index(flat[k]))
            if kind == "ts" and k > 0:
                assert flat[k + 1] >= flat[k] >= st.timestamp_begin
                k += 1
            k += 1
        assert k == len(flat), (k, len(flat))
        assert r.score > -1e-3 and r.no_speech_prob < 1e-6
        choices.append(tuple(pick))
    assert len(set(choices)) >= 2, choices          # the transcript depends on the audio


def test_gates_f32_vs_bf16_oracle(tiny):
    dims, o16, enc, tok, prompt, opt, res = tiny
    g = gate_windows(o16, lambda ws: enc[ws], prompt, res, dims.specials, opt, tok)
    assert_gates(g)
    assert g["identical"] == W and g["min_margin_identical_nats"] > 5.0, g


# ------------------------------------------------------------------------------ variable-length plant (margin_var)
@pytest.fixture(scope="module")
def tiny_var():
    from vlog_amd.weights import plant_margin
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=0)
    plan = plant_margin(sd, dims, 0, variable=True)
    w = round_bf16(sd)
    o32 = OracleWhisper(w, dims, np.float32)
    o16 = OracleWhisper(w, dims, np.float32, bf16_acts=True)
    # windows of the corpus with levels from 8 to -4 (measured): five tokens to ~150; plus window 9 of the
    # variable corpus (room tone: the quiet bit ends it after one token)
    from vlog_amd.audio import long_form_window
    seeds = [10, 0, 3, 4, 12, 1, 2]
    x = np.concatenate([speech_like(30.0, s) for s in seeds] + [long_form_window(9)])
    seeds = seeds + [9]
    n = len(seeds)
    mel = omel.log_mel(x, dims.n_mels)[:, :3000 * n].reshape(dims.n_mels, n, 3000).transpose(1, 0, 2)
    enc = o32.encode(np.ascontiguousarray(mel))
    tok = Tokenizer(dims, language="en")
    prompt = list(tok.sot_sequence)
    opt = GenerateOptions(suppress_tokens=list(tok.suppressed_tokens([-1])), max_length=448)
    res = [generate_one(o32, o32.cross_kv(enc[i:i + 1]), prompt, dims.specials, opt) for i in range(n)]
    return dims, plan, o16, enc, tok, prompt, opt, res


def test_variable_length_follows_the_window_level(tiny_var):
    """The script ends after the first exit timestamp whose threshold the window's level exceeds: lengths from
    1 token to the whole script, each an exact prefix of the planted script (+ its timestamp pairs)."""
    from vlog_amd.weights import QUIET_W, level_weights
    dims, plan, _, enc, _, _, _, res = tiny_var
    LEVEL_W = level_weights(dims.n_mels)
    c, cr = plan.bit_channels
    lengths = []
    quiet = []
    for i, r in enumerate(res):
        bits = np.sign((enc[i][:, c] - enc[i][:, cr]).mean(0))
        s = bits[:6]
        q = int(bits[7]) * plan.quiet_sign                 # +1: the window is silence
        quiet.append(q)
        L = int(sum(w * b for w, b in zip(LEVEL_W, s)))
        k_exit = next((k for e, (k, T) in enumerate(plan.exits) if (QUIET_W * q if e == 0 else L) > T),
                      len(plan.slots) - 1)
        flat, k, pos = list(r.tokens), 0, 0
        while True:                                   # walk the script up to the exit slot
            slot, kind = plan.slots[k], plan.kinds[k]
            assert flat[pos] in slot, (i, pos, flat[pos], slot)
            pos += 1
            if k == k_exit:
                break
            if kind == "ts" and k > 0:
                assert flat[pos] == flat[pos - 1]      # the timestamp pair
                pos += 1
            k += 1
        assert pos == len(flat), (i, L, pos, len(flat))
        assert r.score > -1e-3
        lengths.append((L, len(flat)))
    # the room-tone window is the only quiet one and decodes one token (its first timestamp)
    assert quiet == [-1] * (len(res) - 1) + [1], quiet
    assert lengths[-1][1] == 1, lengths
    # among the speech windows a higher level ends earlier; their levels span five tokens to ~150+
    by_level = sorted(lengths[:-1], key=lambda t: -t[0])
    assert all(a[1] < b[1] for a, b in zip(by_level, by_level[1:]) if a[0] > b[0]), lengths
    assert by_level[0][1] <= 5 and by_level[-1][1] >= 140, lengths


def test_variable_length_gates_f32_vs_bf16_oracle(tiny_var):
    dims, _, o16, enc, tok, prompt, opt, res = tiny_var
    g = gate_windows(o16, lambda ws: enc[ws], prompt, res, dims.specials, opt, tok)
    assert_gates(g)
    assert g["identical"] == len(res) and g["min_margin_identical_nats"] > 5.0, g
