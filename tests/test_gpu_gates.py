"""The north_star parity gates, asserted, on the margin-planted synthetic models (vlog_amd/weights.py plant_margin).

north_star (BASELINE.json): greedy token sequences identical on >= 99 % of windows, WER delta <= 0.3 % absolute,
segment timestamps within one timestamp token (20 ms), identical WebVTT.  On random-init weights these gates
cannot be checked: their logits sit within bf16 noise of each other (tests/test_gpu_configs.py keeps those as
stress tests).  The margin-planted model is decisive like a trained one (top-1 / top-2 gaps of tens to
thousands of nats) and its transcript depends on the audio through window-level bits carried by the encoder.

Every window of every configuration is checked (tests/parity_util.py gate_windows): the GPU's tokens are
teacher-forced through the CPU oracle in the engine's numeric format from the GPU's own encoder output
(identical = the GPU token is the oracle's argmax at every step => the oracle's greedy decode IS the GPU's
sequence); non-identical windows are re-decoded by the oracle's greedy search for WER and segment times.
Reference call: worker/transcription.py:105-131 (segments -> text, start/end -> WebVTT)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle.decode import GenerateOptions, beam_many
from oracle.model import OracleWhisper
from tests.parity_util import GATE_IDENTICAL, assert_gates, gate_windows, sample_indices, source_offset
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu


def _record(name, g):
    p = os.environ.get("VLOG_AMD_PARITY_OUT")
    if p:
        with open(p, "a") as f:
            f.write(json.dumps(dict(name=name, **g)) + "\n")


class MarginConfig:
    def __init__(self, name, n_windows, seed0=0, plant="margin"):
        from vlog_amd.engine import GpuEngine
        self.dims = dims = model_dims(name)
        sd = synthetic_state_dict(dims, seed=0, plant=plant)
        self.eng = GpuEngine(dims, sd, 0)
        self.w = round_bf16(sd)
        del sd
        self.orc = OracleWhisper(self.w, dims, np.float32, bf16_acts=True)
        self.W = n_windows
        # the variable-length model runs on the variable corpus (every 10th window room tone: near-empty windows)
        if plant == "margin_var":
            from vlog_amd.audio import long_form_window
            x = np.concatenate([long_form_window(seed0 + i) for i in range(n_windows)])
        else:
            x = np.concatenate([speech_like(30.0, seed0 + i) for i in range(n_windows)])
        self.audio = x
        self.mel = self.eng.features(torch.from_numpy(x))
        self.enc = self.eng.encode(self.mel, [3000 * i for i in range(n_windows)], [3000] * n_windows)
        self.tok = Tokenizer(dims, language="en")
        self.prompt = list(self.tok.sot_sequence)
        self.sup = list(self.tok.suppressed_tokens([-1]))
        self.st = dims.specials

    def opt(self, beam=1):
        return GenerateOptions(beam_size=beam, suppress_tokens=self.sup, max_length=448)

    def enc_of(self, ws):
        return self.enc[list(ws)].float().cpu().numpy()

    def greedy(self, order=None, **kw):
        """Greedy decode of every window (slots in `order`, default 0..W-1); results by window."""
        order = list(range(self.W)) if order is None else list(order)
        self.eng.reserve(self.W, self.W)
        self.eng.cross_kv(self.enc, 0)
        res, self.steps = self.eng.generate(order, [self.prompt] * self.W, suppress_tokens=self.sup, max_length=448,
                                            check_every=4, **kw)
        out = [None] * self.W
        for w, r in zip(order, res):
            out[w] = r
        return out

    def gates(self, name, res, known=None):
        g = gate_windows(self.orc, self.enc_of, self.prompt, res, self.st, self.opt(), self.tok, known=known)
        g["mean_tokens"] = float(np.mean([len(r.tokens) for r in res]))
        g["distinct_transcripts"] = len({tuple(r.tokens) for r in res})
        _record(name, {k: v for k, v in g.items() if k != "oracle_tokens"})
        return g


def _check(cfg: MarginConfig, name: str):
    res = cfg.greedy()
    assert len(res) == cfg.W
    g = cfg.gates(name, res)
    cfg.oracle_greedy = g["oracle_tokens"]          # the oracle's greedy transcript of every window
    assert_gates(g)
    assert g["distinct_transcripts"] >= 2, g             # the transcript depends on the audio
    assert g["max_no_speech_diff"] < 1e-3, g
    return g


# ------------------------------------------------------------------------------------------ configs 2 and 3
def test_config2_base_32_windows_gates():
    """Config 2: base (multilingual) bf16 greedy, batch 32 x 30 s windows, every window gated."""
    _check(MarginConfig("base", 32), "gates base greedy 32 windows")


def test_config3_small_120_windows_gates():
    """Config 3: small bf16 greedy, 1 h = 120 windows in one batch, every window gated."""
    _check(MarginConfig("small", 120), "gates small greedy 120 windows")


# ------------------------------------------------------------------------------------------ config 4 / 5
@pytest.fixture(scope="module")
def lv3():
    return MarginConfig("large-v3", 150)


def test_config4_large_v3_150_windows_gates(lv3):
    """Config 4 (the bench workload, per GPU): large-v3 bf16 greedy over 150 windows, every window gated."""
    _check(lv3, "gates large-v3 greedy 150 windows")


def test_fp8_cross_memory_gates_vs_bf16_oracle(lv3):
    """Opt-in fp8 (e4m3) cross memory on the same gates, against the FULL-precision oracle
    (the GPU's bf16 encoder output, not the dequantised one): the fp8 mode is gated, not just recorded."""
    lv3.eng.set_option("cross_fp8", 1)
    try:
        res = lv3.greedy()
    finally:
        lv3.eng.set_option("cross_fp8", 0)
    # windows whose fp8 tokens equal the oracle's greedy tokens from the bf16 gate (same encoder output, weights
    # and options) are identical without another oracle pass; the rest are teacher-forced
    g = lv3.gates("gates large-v3 fp8 cross memory 150 windows vs bf16 oracle", res,
                  known=getattr(lv3, "oracle_greedy", None))
    assert_gates(g)


def test_config5_beam5_identical_to_oracle_beam(lv3):
    """Config 5's search: beam 5 over 128 windows (640 hypothesis rows); 5 windows spread over the batch
    re-decoded by the oracle's own beam search (openai BeamSearchDecoder semantics) must give the same
    hypothesis, and the GPU's chosen hypothesis is teacher-forced to the oracle's argmax path."""
    W = 128
    lv3.eng.reserve(150, W * 5)
    lv3.eng.set_option("cross_mode", 0)             # the product's form for beam groups (transcribe.py)
    try:
        lv3.eng.cross_kv(lv3.enc, 0)
        res, _ = lv3.eng.generate(list(range(W)), [lv3.prompt] * W, beam_size=5, patience=1.0,
                                  suppress_tokens=lv3.sup, max_length=448, check_every=4)
    finally:
        lv3.eng.set_option("cross_mode", 1)
    ws = sample_indices(W, 5)
    from tests.parity_util import progress
    progress("beam5: oracle beam search over 5 windows")
    refs = beam_many(lv3.orc, lv3.orc.cross_kv(lv3.enc_of(ws)), lv3.prompt, lv3.st, lv3.opt(beam=5),
                     on_step=lambda pos, nd: pos % 16 == 0 and progress(f"beam5: oracle position {pos}, {nd}/5 windows done"))
    same = [r.tokens == list(res[w].tokens) for w, r in zip(ws, refs)]
    g = gate_windows(lv3.orc, lv3.enc_of, lv3.prompt, res, lv3.st, lv3.opt(beam=5), lv3.tok, windows=ws)
    g.pop("oracle_tokens")
    _record("gates large-v3 beam5 128 windows (5 sampled vs oracle beam)", dict(g, identical_to_oracle_beam=sum(same)))
    assert all(same), (ws, same)
    assert_gates(g)


def test_config5_alignment_large_v3_vs_oracle(lv3):
    """Config 5's word alignment at large-v3 (128 mels, 20 heads, the alignment heads of the last half of the
    decoder): wm_align_batch over 6 windows vs oracle/align.py on the GPU's encoder output — text-token
    probabilities, and the DTW path (jumps) identical on >= 99 % of tokens — in both cross-attention forms: the
    factored one, and the projected one the product runs for beam groups, whose teacher-forced pass takes the
    matrix-core kernel (attn_dec.hip cross_tf_kernel, option cross_tf)."""
    from oracle.align import find_alignment
    st = lv3.st
    res = lv3.greedy()
    ws = sample_indices(lv3.W, 6)
    texts = [[t for t in res[w].tokens if t < st.eot] for w in ws]
    heads = lv3.dims.default_alignment_heads()
    refs = [find_alignment(lv3.orc, lv3.orc.cross_kv(lv3.enc_of([w])), lv3.prompt, text, st, 3000, heads, 7)
            for w, text in zip(ws, texts)]

    def jumps(ti, tj):
        return tj[np.pad(np.diff(ti), (1, 0), constant_values=1).astype(bool)] / 50.0

    try:
        for form, mode in (("factored", 1), ("projected, MFMA teacher-forced pass", 0)):
            lv3.eng.set_option("cross_mode", mode)
            lv3.eng.cross_kv(lv3.enc, 0)
            assert lv3.eng.option("cross_tf") == 1
            got = lv3.eng.align_batch(ws, lv3.prompt, texts, [3000] * len(ws), heads, median_filter_width=7)
            tok_same, tok_total, pmax = 0, 0, 0.0
            for (gp, gi, gj), (rp, ri, rj) in zip(got, refs):
                pmax = max(pmax, float(np.max(np.abs(gp - rp))))
                ja, jr = jumps(gi, gj), jumps(ri, rj)
                assert ja.shape == jr.shape
                tok_same += int(np.sum(np.abs(ja - jr) <= 0.02 + 1e-9))
                tok_total += ja.size
            _record(f"large-v3 alignment vs oracle (6 windows, {form})",
                    dict(tokens_within_20ms=tok_same, tokens=tok_total, max_text_token_prob_diff=pmax))
            assert pmax < 1e-3, form
            assert tok_same >= GATE_IDENTICAL * tok_total, (form, tok_same, tok_total)
    finally:
        lv3.eng.set_option("cross_mode", 1)


# ------------------------------------------------------------------------------------------ config 1
def test_config1_tiny_en_vtt_identical_to_cpu_oracle(tmp_path):
    """Config 1: tiny.en, a 60 s clip -> WebVTT through the worker's call (sequential seek loop, beam 5,
    previous-text prompts), vs the WHOLE path on the CPU oracle (log-mel, encoder and decoder in the engine's
    numeric format, oracle seek loop): byte-identical captions and the same transcript."""
    from oracle import transcribe as otr
    from vlog_amd.audio import load_audio, write_wav
    from vlog_amd.metrics import word_error_rate
    from vlog_amd.transcribe import WhisperModel
    from vlog_amd.vtt import generate_webvtt

    model = WhisperModel("synthetic:tiny.en:0:margin", device="cpu", compute_type="int8")
    x = np.concatenate([speech_like(30.0, 900), speech_like(30.0, 901)])
    wav = tmp_path / "clip.wav"
    write_wav(str(wav), x)
    segs, info = model.transcribe(str(wav), language=None, task="transcribe", beam_size=5, temperature=0.0)
    segs = [dict(start=s.start, end=s.end, text=s.text) for s in segs]
    sd = synthetic_state_dict(model.dims, seed=0, plant="margin")
    orc = OracleWhisper(round_bf16(sd), model.dims, np.float32, bf16_acts=True, bf16_enc=True)
    ref, _ = otr.transcribe(orc, lambda l: Tokenizer(model.dims, language=l), load_audio(str(wav)), beam_size=5,
                            temperatures=(0.0,))
    vtt = generate_webvtt(segs)
    vtt_ref = generate_webvtt([dict(start=r["start"], end=r["end"], text=r["text"]) for r in ref])
    wer = word_error_rate(" ".join(r["text"].strip() for r in ref), " ".join(s["text"].strip() for s in segs))
    _record("gates tiny.en 60 s VTT vs CPU oracle", dict(vtt_identical=vtt == vtt_ref, wer=wer, cues=vtt.count(" --> ")))
    assert vtt == vtt_ref
    assert wer == 0.0 and vtt.count(" --> ") >= 8


# ------------------------------------------------------------------------------------------ variable-length workload
@pytest.fixture(scope="module")
def lv3_var():
    return MarginConfig("large-v3", 150, plant="margin_var")


def test_config4_variable_length_gates_and_row_set_decode(lv3_var):
    """Config 4 on the variable-length planted model (weights.py plant margin_var: the window's audio level picks
    where its script ends: 1 token for the corpus's room-tone windows, 44 to 210 for speech): every window gated against the oracle, with the
    all-rows decode and with the row-set decode the bench runs (windows ordered longest-expected first by
    vlog_amd.shard.expected_tokens, rows refilled as windows end, then compacted), whose tokens must equal the
    all-rows decode's on every window (the model is decisive; the routes differ only in f32 rounding)."""
    from vlog_amd.shard import expected_token_order, expected_tokens
    cfg = lv3_var
    res = cfg.greedy()
    steps_all = cfg.steps
    # every 3rd window plus the shortest and the longest transcript through the oracle (every window of the uniform
    # config 4 is gated above; VLOG_AMD_GATE_STRIDE=1 gates every window here too)
    stride = max(1, int(os.environ.get("VLOG_AMD_GATE_STRIDE", "3")))
    offset = source_offset(stride, "VLOG_AMD_GATE_OFFSET")           # 0 unless pinned or VLOG_AMD_SWEEP_ROTATE=1
    lens0 = [len(r.tokens) for r in res]
    gw = sorted(set(range(offset, cfg.W, stride)) | {int(np.argmin(lens0)), int(np.argmax(lens0))})
    g = gate_windows(cfg.orc, cfg.enc_of, cfg.prompt, res, cfg.st, cfg.opt(), cfg.tok, windows=gw)
    g.pop("oracle_tokens", None)
    _record(f"gates large-v3 variable-length greedy 150 windows ({len(gw)} gated)",
            dict({k: v for k, v in g.items()}, stride=stride, offset=offset))
    assert_gates(g)
    lens = [len(r.tokens) for r in res]
    # the corpus's 150 windows: the 15 room-tone windows decode one token (the quiet bit), the speech windows 44 to
    # 210 under plant margin_var's level orientation
    assert min(lens) <= 5 and max(lens) >= 170 and 60 <= float(np.mean(lens)) <= 160, sorted(lens)
    assert sum(n <= 5 for n in lens) >= cfg.W // 10, sorted(lens)
    db = cfg.eng.frame_energy_db(torch.from_numpy(cfg.audio), 512)
    expect = expected_tokens(db, 512, [480000 * i for i in range(cfg.W)], [480000] * cfg.W)
    order = expected_token_order(expect)
    corr = float(np.corrcoef(expect, lens)[0, 1])
    st = {}
    rows = cfg.greedy(order=order, max_rows=112, compact=True, stats=st)
    same = sum(a.tokens == b.tokens for a, b in zip(res, rows))
    _record("row-set decode large-v3 variable-length 150 windows", dict(
        same_tokens=same, stats=st, steps_all_rows=steps_all, mean_tokens=float(np.mean(lens)),
        expected_vs_actual_tokens_corr=corr,
        lengths_min_max=(min(lens), max(lens)),
        active_row_fraction_all_rows=float(sum(n + 1 for n in lens) / (steps_all * cfg.W)),
        active_row_fraction_row_set=float(sum(n + 1 for n in lens) / max(1, st["row_steps"]))))
    assert same == cfg.W, same


def test_config5_beam_compaction_variable_length(lv3_var):
    """Config 5's search on the variable-length model: beam 5 over 60 windows with the hypotheses of finished
    windows dropped from the passes (wm_generate compact, beam) vs the all-rows beam decode: the same hypothesis
    on every window (the model is decisive; the routes differ only in f32 rounding), scores within f32 rounding,
    and fewer row-steps; 4 windows re-decoded by the oracle's own beam search."""
    cfg = lv3_var
    W = 60
    cfg.eng.reserve(cfg.W, W * 5)
    cfg.eng.set_option("cross_mode", 0)             # the product's form for beam groups (transcribe.py)
    try:
        cfg.eng.cross_kv(cfg.enc, 0)
        out = {}
        for compact in (False, True):
            st = {}
            res, steps = cfg.eng.generate(list(range(W)), [cfg.prompt] * W, beam_size=5, patience=1.0,
                                          suppress_tokens=cfg.sup, max_length=448, check_every=4, compact=compact,
                                          stats=st)
            out[compact] = (res, steps, st)
        # the beam row-set decode (engine.cpp generate_rows_beam): 20 windows' groups in flight, a finished window's
        # group taking the next one (windows in reverse order, so long and short ones mix), then compaction
        order = list(range(W))[::-1]
        st_rows = {}
        res_rows, _ = cfg.eng.generate(order, [cfg.prompt] * W, beam_size=5, patience=1.0, suppress_tokens=cfg.sup,
                                       max_length=448, check_every=4, max_rows=100, compact=True, stats=st_rows)
        rc = [None] * W
        for w, r in zip(order, res_rows):
            rc[w] = r
    finally:
        cfg.eng.set_option("cross_mode", 1)
    (ra, sa, ta), (rb, sb, tb) = out[False], out[True]
    same_rows = sum(a.tokens == b.tokens for a, b in zip(ra, rc))
    _record("beam5 row-set decode (20 groups) large-v3 variable-length 60 windows",
            dict(same_tokens=same_rows, stats=st_rows, all_rows_row_steps=ta["row_steps"]))
    assert same_rows == W, same_rows
    assert st_rows["refills"] == W - 20, st_rows
    for a, b in zip(ra, rc):
        assert abs(a.score - b.score) <= 1e-3 * max(1.0, abs(a.score))
        assert abs(a.no_speech_prob - b.no_speech_prob) < 1e-4
    same = sum(a.tokens == b.tokens for a, b in zip(ra, rb))
    lens = [len(r.tokens) for r in ra]
    lens0 = [len(r.tokens) for r in ra]
    ws = [int(np.argmin(lens0)), int(np.argmax(lens0))]     # the shortest and the longest transcript
    refs = beam_many(cfg.orc, cfg.orc.cross_kv(cfg.enc_of(ws)), cfg.prompt, cfg.st, cfg.opt(beam=5))
    oracle_same = sum(r.tokens == list(rb[w].tokens) for w, r in zip(ws, refs))
    _record("beam5 compaction large-v3 variable-length 60 windows", dict(
        same_tokens=same, oracle_beam_identical=oracle_same, steps=(sa, sb), row_steps=(ta["row_steps"], tb["row_steps"]),
        lengths_min_max=(min(lens), max(lens))))
    assert same == W, same
    assert oracle_same == len(ws), oracle_same
    for a, b in zip(ra, rb):
        assert abs(a.score - b.score) <= 1e-3 * max(1.0, abs(a.score))
        assert abs(a.no_speech_prob - b.no_speech_prob) < 1e-4
    assert tb["row_steps"] < ta["row_steps"], (ta, tb)
