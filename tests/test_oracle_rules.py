"""Timestamp logit rules (oracle/decode.py apply_rules) pinned against transformers
WhisperTimeStampLogitsProcessor ([TF] generation/logits_process.py:1909-2049) on crafted histories."""
import numpy as np
import pytest
import torch
from transformers import GenerationConfig
from transformers.generation.logits_process import WhisperTimeStampLogitsProcessor

from oracle.decode import apply_rules
from vlog_amd.dims import model_dims

ST = model_dims("large-v3").specials
TB = ST.timestamp_begin
PROMPT = [ST.sot, ST.lang_token("en"), ST.transcribe]

HISTORIES = [
    [], [TB + 10], [TB + 10, 500], [TB + 10, 500, TB + 40], [TB + 10, 500, TB + 40, TB + 40],
    [TB + 10, 500, 600, TB + 90, TB + 90, 700], [TB, TB], [TB + 3, 17, TB + 1500],
    [TB + 1499, 9, 10, 11], [TB + 5, 8, TB + 6, TB + 6, 42, 43],
]


def _hf(history, logits, mit):
    gc = GenerationConfig(eos_token_id=ST.eot, no_timestamps_token_id=ST.no_timestamps, max_initial_timestamp_index=mit)
    proc = WhisperTimeStampLogitsProcessor(gc, begin_index=len(PROMPT))
    ids = torch.tensor([PROMPT + history])
    return proc(ids, torch.from_numpy(logits[None].astype(np.float32)))[0].numpy()


@pytest.mark.parametrize("hi", range(len(HISTORIES)))
@pytest.mark.parametrize("scale", [0.5, 4.0])
def test_timestamp_rules_match_transformers(hi, scale):
    rng = np.random.default_rng(hi)
    logits = (rng.standard_normal(51866) * scale).astype(np.float32)
    logits[TB:] += rng.standard_normal(51866 - TB) * scale - 2.0
    hist = HISTORIES[hi]
    got = apply_rules(logits, hist, ST, (), False, 50)
    ref = _hf(hist, logits, 50)
    assert np.array_equal(np.isinf(got), np.isinf(ref))
    fin = np.isfinite(ref)
    assert np.allclose(got[fin], ref[fin], atol=1e-5)


def test_suppress_blank_and_tokens_first_step():
    logits = np.zeros(51866, dtype=np.float32)
    got = apply_rules(logits, [], ST, (5, 7), True, 50, with_timestamps=False)
    assert np.isinf(got[[ST.blank, ST.eot, 5, 7]]).all() and np.isfinite(got[8])


def test_gumbel_noise_is_finite_gumbel():
    """The counter-based sampling noise (oracle restatement of the engine's): finite for every counter (u stays
    strictly inside (0, 1)), Gumbel-distributed, and a pure function of (seed, hypothesis, step, token)."""
    from oracle.decode import gumbel_noise
    import numpy as np
    g = np.concatenate([gumbel_noise(s, h, t, 51866) for s in (0, 7) for h in (0, 5) for t in (0, 3, 400)])
    assert np.all(np.isfinite(g))
    assert abs(float(g.mean()) - 0.5772) < 0.01 and abs(float(g.std()) - 1.2825) < 0.02
    assert np.array_equal(gumbel_noise(7, 5, 3, 100), gumbel_noise(7, 5, 3, 1000)[:100])
