"""Beam search, sampling, language detection, word alignment and end-to-end transcribe on the MI355X vs the
CPU oracle (identical encoder outputs at the generate/align boundary; identical audio end to end)."""
import numpy as np
import pytest
import torch

from oracle import mel as omel
from oracle import transcribe as otr
from oracle.align import dtw, find_alignment
from oracle.decode import GenerateOptions, detect_language, generate_one
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like
from vlog_amd.dims import model_dims
from vlog_amd.metrics import word_error_rate
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import round_bf16, synthetic_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=3, eot_after=60)
    eng = GpuEngine(dims, sd, 0)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32)
    orc.bf = OracleWhisper(round_bf16(sd), dims, np.float32, bf16_acts=True)   # engine numeric format (decoder)
    W = 4
    x = np.concatenate([speech_like(30.0, 200 + i) for i in range(W)])
    feats = omel.log_mel(x, dims.n_mels)
    enc = eng.encode(torch.from_numpy(feats).cuda(), [3000 * i for i in range(W)], [3000] * W)
    eng.reserve(W, 40)
    eng.cross_kv(enc, 0)
    return dims, eng, orc, enc.float().cpu().numpy(), W


def _sup(st):
    return [st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm]


EPS = 0.02   # nats, the bf16 logit noise floor


def test_beam_search_matches_oracle(setup):
    """Beam 5 / patience 1: the GPU's chosen hypothesis, scored by the oracle, must be EPS-optimal against the
    oracle's own beam result, and every token must be rule-legal; most windows are identical outright."""
    from oracle.decode import score_sequence
    dims, eng, orc, encf, W = setup
    st = dims.specials
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    opt = GenerateOptions(beam_size=5, suppress_tokens=_sup(st), max_length=100)
    res, _ = eng.generate(list(range(W)), [prompt] * W, beam_size=5, patience=1.0, suppress_tokens=_sup(st), max_length=100)
    same = 0
    for w in range(W):
        cross = orc.cross_kv(encf[w: w + 1])
        r = generate_one(orc, cross, prompt, st, opt)
        same += r.tokens == res[w].tokens
        ended = len(prompt) + len(res[w].tokens) < 100
        chosen, best, score = score_sequence(orc, cross, prompt, res[w].tokens, st, opt, ended)
        assert np.all(np.isfinite(chosen))                       # every token allowed by the rules
        assert score >= r.score - EPS, (score, r.score)
        assert abs(score - res[w].score) < 2e-2 * max(1.0, abs(score))
    assert same >= W - 1, f"{same}/{W}"


def test_sampling_obeys_timestamp_rules(setup):
    dims, eng, orc, encf, W = setup
    st = dims.specials
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    res, _ = eng.generate(list(range(W)), [prompt] * W, temperature=1.0, num_hypotheses=3, seed=7,
                          suppress_tokens=_sup(st), max_length=120)
    res2, _ = eng.generate(list(range(W)), [prompt] * W, temperature=1.0, num_hypotheses=3, seed=7,
                           suppress_tokens=_sup(st), max_length=120)
    tb = st.timestamp_begin
    for r, r2 in zip(res, res2):
        assert r.tokens == r2.tokens                          # seeded -> reproducible
        assert r.tokens and tb <= r.tokens[0] <= tb + 50      # first token: timestamp <= 1.00 s
        ts = [t for t in r.tokens if t >= tb]
        assert ts == sorted(ts)                               # monotonic timestamps
        assert not (set(r.tokens) & set(_sup(st)))


def test_prompted_generate_matches_oracle(setup):
    """Previous-text conditioning (faster-whisper get_prompt): <|startofprev|> + history + sot sequence."""
    dims, eng, orc, encf, W = setup
    st = dims.specials
    prompt = [st.sot_prev] + list(range(400, 460)) + [st.sot, st.lang_token("en"), st.transcribe]
    res, _ = eng.generate([1], [prompt], suppress_tokens=_sup(st), max_length=160)
    from oracle.decode import score_sequence
    opt = GenerateOptions(suppress_tokens=_sup(st), max_length=160)
    cross = orc.cross_kv(encf[1:2])
    r = generate_one(orc, cross, prompt, st, opt)
    chosen, best, _ = score_sequence(orc, cross, prompt, res[0].tokens, st, opt, len(prompt) + len(res[0].tokens) < 160)
    assert r.tokens == res[0].tokens or np.all(chosen >= best - EPS)
    assert abs(r.no_speech_prob - res[0].no_speech_prob) < 1e-3


def test_detect_language_matches_oracle(setup):
    dims, eng, orc, encf, W = setup
    st = dims.specials
    logits, _ = eng.forward([2], np.array([[st.sot]]), last_only=True)
    p = torch.softmax(logits[0, st.lang_begin: st.lang_begin + st.n_langs].double(), 0).cpu().numpy()
    ref = detect_language(orc, orc.cross_kv(encf[2:3]), st)
    assert st.lang_codes[int(np.argmax(p))] == ref[0][0]
    assert abs(p.max() - ref[0][1]) < 5e-3


@pytest.mark.parametrize("shape", [(1, 1), (5, 17), (30, 400), (120, 1500)])
def test_dtw_kernel_matches_oracle(setup, shape):
    _, eng, _, _, _ = setup
    x = np.random.default_rng(shape[0]).standard_normal(shape).astype(np.float32)
    gi, gj = eng.dtw(torch.from_numpy(x))
    ri, rj = dtw(x.astype(np.float64).astype(np.float32))
    assert np.array_equal(gi, ri) and np.array_equal(gj, rj)


def _jumps(ti, tj):
    return tj[np.pad(np.diff(ti), (1, 0), constant_values=1).astype(bool)]


def test_alignment_attention_capture(setup):
    """Cross-attention weights of the alignment heads captured by wm_forward vs the oracle (bf16 tolerance)."""
    dims, eng, orc, encf, W = setup
    st = dims.specials
    tok = Tokenizer(dims, language="en")
    toks = tok.sot_sequence + [st.no_timestamps] + list(range(1000, 1040)) + [st.eot]
    heads = dims.default_alignment_heads()
    _, attn = eng.forward([3], np.array([toks]), align_heads=heads)
    _, _, cw = orc.decode(np.array([toks]), orc.cross_kv(encf[3:4]), return_cross_attn=True)
    ref = np.stack([cw[l][0, h] for l, h in heads], 1)            # [S, heads, 1500]
    got = attn[0].cpu().numpy()
    assert np.abs(got - ref).max() < 2e-3
    assert np.allclose(got.sum(-1), 1.0, atol=1e-4)


def test_alignment_postprocess_matches_oracle(setup):
    """GPU normalise + median filter + DTW on the SAME captured attention as the oracle post-processing."""
    from oracle.align import alignment_matrix
    dims, eng, orc, encf, W = setup
    st = dims.specials
    tok = Tokenizer(dims, language="en")
    text = list(range(1000, 1040))
    heads = dims.default_alignment_heads()
    toks = tok.sot_sequence + [st.no_timestamps] + text + [st.eot]
    _, attn = eng.forward([3], np.array([toks]), align_heads=heads)
    probs, ti, tj = eng.align(3, tok.sot_sequence, text, 3000, heads, 7)
    m = alignment_matrix(attn[0].cpu().numpy().transpose(1, 0, 2), 3000, len(tok.sot_sequence))
    ri, rj = dtw(-m)
    jg, jr = _jumps(ti, tj), _jumps(ri, rj)
    assert len(jg) == len(jr) and np.mean(jg == jr) >= 0.97


def _align_vs_oracle(eng, orc, encf, dims, slot):
    st = dims.specials
    tok = Tokenizer(dims, language="en")
    text = list(range(1000, 1040))
    heads = dims.default_alignment_heads()
    probs, ti, tj = eng.align(slot, tok.sot_sequence, text, 3000, heads, 7)
    rp, ri, rj = find_alignment(orc, orc.cross_kv(encf[slot:slot + 1]), tok.sot_sequence, text, st, 3000, heads)
    assert np.allclose(probs, rp, rtol=0.05, atol=1e-6)
    jg, jr = _jumps(ti, tj), _jumps(ri, rj)
    assert len(jg) == len(jr)
    return float(np.mean(np.abs(jg - jr) <= 1))


def test_word_alignment_end_to_end_vs_oracle(setup):
    """Whole align (bf16 decoder) vs the float32 oracle on the synthetic model.  Its cross-attention is nearly
    uniform, so DTW near-ties move the path tail under any bf16 noise: the projected (cross_mode 0) and the
    factored form (default) carry score errors of the same size and land at 0.85-0.93 of
    token start times within 20 ms depending on the noise draw; this checks both stay in that band.  The
    well-conditioned bar is the sharpened-attention test below."""
    dims, eng, orc, encf, W = setup
    enc = torch.from_numpy(encf).to(torch.bfloat16).cuda()
    frac = {}
    for mode in (0, 1):
        eng.set_option("cross_mode", mode)
        eng.cross_kv(enc, 0)
        frac[mode] = _align_vs_oracle(eng, orc, encf, dims, 3)
    assert min(frac.values()) >= 0.80, frac


def test_word_alignment_sharpened_attention_vs_oracle():
    """The same end-to-end alignment on a model whose alignment-layer cross-attention queries are scaled by 6
    (peaked attention, as a trained model's alignment heads): fewer DTW near-ties, so a tighter bar — >= 90 %
    of token start times within 20 ms of the oracle in both cross-attention forms, per window."""
    from vlog_amd.engine import GpuEngine
    dims = model_dims("tiny")
    sd = synthetic_state_dict(dims, seed=3, eot_after=60)
    for l in sorted({l for l, _ in dims.default_alignment_heads()}):
        p = f"model.decoder.layers.{l}.encoder_attn.q_proj."
        sd[p + "weight"] = sd[p + "weight"] * 6.0
        sd[p + "bias"] = sd[p + "bias"] * 6.0
    eng = GpuEngine(dims, sd, 0)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32)
    x = np.concatenate([speech_like(30.0, 200 + i) for i in range(2)])
    feats = omel.log_mel(x, dims.n_mels)
    enc = eng.encode(torch.from_numpy(feats).cuda(), [0, 3000], [3000, 3000])
    eng.reserve(2, 4)
    encf = enc.float().cpu().numpy()
    frac = {}
    for mode in (0, 1):
        eng.set_option("cross_mode", mode)
        eng.cross_kv(enc, 0)
        frac[mode] = [_align_vs_oracle(eng, orc, encf, dims, slot) for slot in (0, 1)]
    assert min(min(v) for v in frac.values()) >= 0.90, frac


class _GpuBackend:
    """The GPU engine behind the oracle's seek loop: both host loops then share one decoder, so their
    segments must agree exactly (decoder numerics are covered by the epsilon-consistency tests)."""

    def __init__(self, model):
        self.m = model

    def encode(self, window):
        enc = self.m.engine.encode(torch.from_numpy(np.ascontiguousarray(window, dtype=np.float32)).cuda(), [0], [3000])
        self.m.engine.cross_kv(enc, 0)
        return 0

    def generate(self, slot, prompt, opt):
        from oracle.decode import GenerateResult
        st = self.m.dims.specials
        res, _ = self.m.engine.generate([slot], [prompt], beam_size=opt.beam_size, patience=opt.patience,
                                        length_penalty=opt.length_penalty, max_length=opt.max_length,
                                        suppress_tokens=opt.suppress_tokens, suppress_blank=opt.suppress_blank,
                                        max_initial_timestamp_index=opt.max_initial_timestamp_index,
                                        sot_index=prompt.index(st.sot))
        r = res[0]
        return GenerateResult(r.tokens, r.score, r.no_speech_prob, r.cum_logprob)

    def detect_language(self, slot):
        st = self.m.dims.specials
        logits, _ = self.m.engine.forward([slot], np.array([[st.sot]]), last_only=True)
        p = torch.softmax(logits[0, st.lang_begin: st.lang_begin + st.n_langs].double(), 0).cpu().numpy()
        order = np.argsort(-p, kind="stable")
        return [(st.lang_codes[i], float(p[i])) for i in order]


def test_transcribe_host_loop_matches_oracle(tmp_path):
    """vlog_amd.WhisperModel.transcribe (faster-whisper seek loop: prompts, splitting, skip logic) vs
    oracle/transcribe.py on the SAME decoder: segments must be identical."""
    from vlog_amd.audio import load_audio, write_wav
    from vlog_amd.transcribe import WhisperModel
    model = WhisperModel("synthetic:tiny:3", device="cpu", compute_type="int8", eot_after=60)  # worker's args
    x = np.concatenate([speech_like(30.0, 300), speech_like(25.0, 301), speech_like(14.0, 302)])
    wav = tmp_path / "clip.wav"
    write_wav(str(wav), x)
    # temperature 0 only: the random model's avg log-prob (~ -7) would otherwise trigger the sampled fallback
    # temperatures on every window, whose RNG streams legitimately differ between the loops
    segs, info = model.transcribe(str(wav), language=None, task="transcribe", beam_size=5, temperature=0.0)
    segs = list(segs)
    assert len(segs) > 3 and all(s.temperature == 0.0 for s in segs)
    pcm = load_audio(str(wav))
    feats = model.engine.features(torch.from_numpy(pcm)).cpu().numpy()
    assert np.abs(feats - omel.log_mel(pcm, model.dims.n_mels)).max() <= 1e-4
    ref, lang = otr.transcribe(_Dims(model.dims), lambda l: Tokenizer(model.dims, language=l), pcm,
                               beam_size=5, temperatures=(0.0,), features=feats, backend=_GpuBackend(model))
    assert info.language == lang
    assert [s.tokens for s in segs] == [r["tokens"] for r in ref]
    assert word_error_rate(" ".join(r["text"] for r in ref), " ".join(s.text for s in segs)) == 0.0
    for s, r in zip(segs, ref):
        assert abs(s.start - r["start"]) < 1e-9 and abs(s.end - r["end"]) < 1e-9


class _Dims:
    def __init__(self, dims):
        self.dims = dims


def test_transcribe_fallback_policy_runs():
    """Default temperatures: windows whose avg log-prob is below -1 are re-decoded at rising temperatures
    (faster-whisper generate_with_fallback); the random model fails every threshold, so the last
    temperature is reported and the best below-compression-threshold result is kept."""
    from vlog_amd.transcribe import WhisperModel
    model = WhisperModel("synthetic:tiny:3", device="cuda", eot_after=60)
    x = np.concatenate([speech_like(30.0, 310), speech_like(12.0, 311)])
    segs, info = model.transcribe(x, language="en", beam_size=5)
    segs = list(segs)
    assert segs and all(s.temperature == 1.0 for s in segs)
    assert all(s.avg_logprob < -1.0 and s.compression_ratio <= 2.4 for s in segs)
    assert [s.id for s in segs] == list(range(1, len(segs) + 1))
    assert all(a.end <= b.start + 1e-9 or a.seek != b.seek for a, b in zip(segs, segs[1:]))


def test_worker_call_pattern_and_vtt(tmp_path):
    """The reference worker's exact calls (worker/transcription.py:81-85, 105-131) through the compat
    overlay, then the worker's WebVTT format (vlog_amd.vtt == reference generate_webvtt, goldens)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "compat"))
    from faster_whisper import WhisperModel as FWModel
    from vlog_amd.audio import write_wav
    from vlog_amd.vtt import generate_webvtt
    model = FWModel("synthetic:tiny:3", device="cpu", compute_type="int8", eot_after=60)
    wav = tmp_path / "a.wav"
    write_wav(str(wav), np.concatenate([speech_like(30.0, 320), speech_like(9.0, 321)]))
    segments, info = model.transcribe(str(wav), language=None, task="transcribe", beam_size=5, vad_filter=True)
    seg_list, parts = [], []
    for s in segments:
        seg_list.append({"start": s.start, "end": s.end, "text": s.text})
        parts.append(s.text.strip())
    result = {"text": " ".join(parts), "language": info.language, "segments": seg_list}
    assert isinstance(result["language"], str) and len(result["language"]) <= 10
    vtt = generate_webvtt(result["segments"])
    assert vtt.startswith("WEBVTT\n\n")
    assert vtt.count(" --> ") == len(seg_list)
    assert info.duration_after_vad <= info.duration


def test_vad_filter_drops_long_silence():
    """vad_filter=True (the worker's call): a 6 s silence between two speech clips is removed before decoding
    and segment times are mapped back to the original timeline."""
    from vlog_amd.transcribe import WhisperModel
    model = WhisperModel("synthetic:tiny:3", device="cuda", eot_after=60)
    a, b = speech_like(12.0, 330), speech_like(10.0, 331)
    x = np.concatenate([a, np.zeros(16000 * 6, np.float32), b])
    segs, info = model.transcribe(x, language="en", beam_size=1, temperature=0.0, vad_filter=True)
    segs = list(segs)
    assert info.duration_after_vad < info.duration - 3.0
    # the contract (faster-whisper transcribe with vad_filter): decode the collected speech, then map every
    # segment time back through the speech map.  (Ends are not clamped to the audio: on a random-weight model a
    # window's last timestamp may exceed its content, as in faster-whisper.)
    from vlog_amd.transcribe import VadOptions
    from vlog_amd.vad import SpeechTimestampsMap, collect_chunks, get_speech_timestamps
    chunks = get_speech_timestamps(x, VadOptions(), model)
    assert len(chunks) == 2 and chunks[0]["end"] <= 12 * 16000 + 16000 and chunks[1]["start"] >= 17 * 16000
    plain, _ = model.transcribe(collect_chunks(x, chunks), language="en", beam_size=1, temperature=0.0)
    plain = list(plain)
    m = SpeechTimestampsMap(chunks, 16000)
    assert [s.tokens for s in segs] == [p.tokens for p in plain] and segs
    for s, p in zip(segs, plain):
        assert s.start == m.get_original_time(p.start) and s.end == m.get_original_time(p.end, is_end=True)
        assert 0.0 <= s.start <= s.end


def test_batched_pipeline_matches_single_window_decode():
    """BatchedInferencePipeline (throughput mode): batching windows (two batches of up to 4) gives exactly the
    tokens of one-window generate calls with the same prompt; transcribe() yields their segments in order."""
    from vlog_amd.transcribe import BatchedInferencePipeline, WhisperModel, default_batched_options, TranscriptionOptions
    model = WhisperModel("synthetic:tiny:3", device="cuda", eot_after=60)
    x = np.concatenate([speech_like(30.0, 340 + i) for i in range(5)] + [speech_like(7.0, 345)])
    pipe = BatchedInferencePipeline(model, max_batch_windows=4)
    feats = model.engine.features(torch.from_numpy(x))
    tok = model.tokenizer(language="en")
    opts = TranscriptionOptions(**default_batched_options(beam_size=1, temperature=0.0))
    opts.suppress_tokens = list(tok.suppressed_tokens([-1]))
    wins = pipe.fixed_windows(feats.shape[1] - 1)
    results = pipe.decode_windows(feats, wins, [s * 0.01 for s, _ in wins], tok, opts)
    assert len(results) == 6 and wins[-1][1] == 700
    # greedy: the batched call chose the factored cross-attention form (transcribe.py _use_cross_form), the
    # engine's default, which the single-window calls below use too
    for (seek, size), wr in zip(wins, results):
        enc = model.engine.encode(feats, [seek], [size])
        model.engine.cross_kv(enc, 0)
        res, _ = model.engine.generate([0], [tok.sot_sequence], suppress_tokens=opts.suppress_tokens, max_length=448)
        assert wr.tokens == res[0].tokens
    segs, info = pipe.transcribe(x, language="en", beam_size=1, temperature=0.0, vad_filter=False,
                                 without_timestamps=False)
    segs = list(segs)
    assert segs and all(a.start <= b.start for a, b in zip(segs, segs[1:]))


def test_sharded_transcriber_two_processes():
    """Spawn-based window sharding (vlog_amd.shard.ShardedTranscriber): two worker processes (here both on
    GPU 0) produce the same segments as one worker."""
    import subprocess
    import sys
    code = r'''
import sys, json, numpy as np
sys.path.insert(0, "ROOT")
from vlog_amd.audio import speech_like
from vlog_amd.shard import ShardedTranscriber
x = np.concatenate([speech_like(30.0, 350 + i) for i in range(3)] + [speech_like(13.0, 353)])
out = {}
for devs in ([0], [0, 0]):
    st = ShardedTranscriber("synthetic:tiny:3", devices=devs, eot_after=60)
    segs = st.transcribe(x, language="en", beam_size=1, temperature=0.0)
    st.close()
    out[len(devs)] = [(round(s["start"], 3), round(s["end"], 3), s["tokens"]) for s in segs]
print(json.dumps(out))
'''
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code.replace("ROOT", root)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["1"] == out["2"] and len(out["1"]) > 0


def test_worker_call_throughput_mode(tmp_path, monkeypatch):
    """VLOG_AMD_THROUGHPUT=1: the unchanged worker's call (compat overlay, vad_filter=True, beam 5) runs through
    BatchedInferencePipeline and still yields timed segments for its WebVTT; on a clip without long pauses the
    windows are the same 30 s windows, so the text matches the batched pipeline called directly."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "compat"))
    from faster_whisper import WhisperModel as FWModel
    from vlog_amd.audio import write_wav
    from vlog_amd.transcribe import BatchedInferencePipeline
    from vlog_amd.vtt import generate_webvtt
    monkeypatch.setenv("VLOG_AMD_THROUGHPUT", "1")
    model = FWModel("synthetic:tiny:3", device="cpu", compute_type="int8", eot_after=60)
    assert model.throughput
    wav = tmp_path / "t.wav"
    x = np.concatenate([speech_like(30.0, 360 + i) for i in range(3)])
    write_wav(str(wav), x)
    segments, info = model.transcribe(str(wav), language=None, task="transcribe", beam_size=5, vad_filter=True,
                                      temperature=0.0)
    seg_list = [{"start": s.start, "end": s.end, "text": s.text} for s in segments]
    vtt = generate_webvtt(seg_list)
    assert seg_list and vtt.count(" --> ") == len(seg_list)
    direct, _ = BatchedInferencePipeline(model).transcribe(str(wav), language=info.language, beam_size=5, vad_filter=True,
                                                           temperature=0.0, without_timestamps=False)
    assert [s["text"] for s in seg_list] == [s.text for s in direct]
