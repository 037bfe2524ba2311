"""CPU: the product's word-timestamp host logic (vlog_amd/transcribe.py find_alignment tail,
add_word_timestamps, merge_punctuations) vs oracle/transcribe.py's independent restatement, on seeded
synthetic alignments (a fake engine stands in for wm_align_batch; no GPU needed)."""
import numpy as np
import pytest

from oracle import transcribe as otr
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.transcribe import WhisperModel


class _FakeEngine:
    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)
        self.calls = []

    def align_batch(self, slots, sot, texts, frames, heads, medw):
        out = []
        for t, f in zip(texts, frames):
            n, F = len(t) + 1, f // 2
            # a monotone DTW-like path: text index non-decreasing, time index non-decreasing
            steps = ["d"] * min(n, F) + ["t"] * (F - min(n, F)) + ["i"] * (n - min(n, F))
            self.rng.shuffle(steps)
            i = j = 0
            ti, tj = [0], [0]
            for s in steps[1:]:
                if s == "d" or (s == "t" and j == F - 1) or (s == "i" and i == n - 1):
                    i, j = min(i + 1, n - 1), min(j + 1, F - 1)
                elif s == "t":
                    j += 1
                else:
                    i += 1
                ti.append(i)
                tj.append(j)
            out.append((self.rng.uniform(0.05, 1.0, len(t)).astype(np.float32), np.array(ti), np.array(tj)))
            self.calls.append(len(t))
        return out


def _model(seed):
    m = WhisperModel.__new__(WhisperModel)
    m.dims = model_dims("tiny")
    m.engine = _FakeEngine(seed)
    m.frames_per_second, m.tokens_per_second = 100, 50
    return m


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_add_word_timestamps_matches_oracle_restatement(seed):
    m = _model(seed)
    tok = Tokenizer(m.dims, language="en")
    rng = np.random.default_rng(100 + seed)
    tb = tok.timestamp_begin
    groups, aligns = [], []
    last = 0.0
    for g in range(3):                                  # three windows, several segments each
        seek = 3000 * g
        segs_, t0 = [], 0
        for _ in range(int(rng.integers(1, 4))):
            n = int(rng.integers(1, 12))
            body = [int(v) for v in rng.integers(200, 20000, n)]
            if rng.random() < 0.3:                      # punctuation tokens exercise merge_punctuations
                body[int(rng.integers(0, n))] = tok.encode(",")[0]
            t1 = t0 + int(rng.integers(5, 200))
            segs_.append(dict(seek=seek, start=seek / 100 + t0 * 0.02, end=seek / 100 + t1 * 0.02,
                              tokens=[tb + t0] + body + [tb + t1]))
            t0 = t1
        groups.append(segs_)
    import copy
    prod = copy.deepcopy(groups)
    last_p = m.add_word_timestamps(prod, tok, [3000, 2400, 3000], "\"'“¿([{-", "\"'.。,，!！?？:：”)]}、", 0.0,
                                   slots=[0, 1, 2])
    # oracle: the same alignments (replayed from the fake engine's draws)
    m2 = _model(seed)
    ref = copy.deepcopy(groups)
    texts = [[t for s in g for t in s["tokens"] if t < tok.eot] for g in ref]
    al = m2.engine.align_batch([0, 1, 2], tok.sot_sequence, texts, [3000, 2400, 3000], None, 7)
    aligns = [otr.words_from_alignment(tok, t, p, i, j) for t, (p, i, j) in zip(texts, al)]
    last_r = otr.add_word_timestamps(ref, tok, aligns, 0.0)
    assert last_p == last_r
    for gp, gr in zip(prod, ref):
        for sp, sr in zip(gp, gr):
            assert (sp["start"], sp["end"]) == (sr["start"], sr["end"])
            assert [(w["word"], w["start"], w["end"], float(w["probability"])) for w in sp["words"]] == \
                   [(w["word"], w["start"], w["end"], float(w["probability"])) for w in sr["words"]]
    assert m.engine.calls == [len(t) for t in texts]    # one batched align call for the three windows
