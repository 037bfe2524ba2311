"""Host segment logic (faster-whisper _split_segments_by_timestamps / fallback policy) — known-answer tests."""
from vlog_amd.segments import avg_logprob, compression_ratio, needs_fallback, should_skip_window, split_segments_by_timestamps

TB = 50365


def test_pairs_and_unfinished_tail():
    toks = [TB + 0, 100, 101, TB + 50, TB + 50, 102, TB + 120, TB + 120, 103]
    segs, seek, single = split_segments_by_timestamps(toks, TB, 10.0, 3000, 30.0, 1000)
    assert not single
    assert [(s["start"], s["end"]) for s in segs] == [(10.0, 11.0), (11.0, 12.4)]
    assert segs[0]["tokens"] == [TB, 100, 101, TB + 50]
    assert seek == 1000 + 120 * 2                     # seek to the last complete timestamp


def test_single_timestamp_ending_consumes_window():
    toks = [TB + 0, 100, TB + 25, TB + 25, 101, TB + 80]
    segs, seek, single = split_segments_by_timestamps(toks, TB, 0.0, 3000, 30.0, 0)
    assert single and seek == 3000
    assert [(round(s["start"], 6), round(s["end"], 6)) for s in segs] == [(0.0, 0.5), (0.5, 1.6)]


def test_no_consecutive_timestamps():
    segs, seek, _ = split_segments_by_timestamps([TB + 3, 5, 6, TB + 40], TB, 30.0, 2000, 20.0, 3000)
    assert len(segs) == 1 and segs[0]["start"] == 30.0 and abs(segs[0]["end"] - 30.8) < 1e-9
    assert seek == 5000
    segs, _, _ = split_segments_by_timestamps([5, 6], TB, 0.0, 3000, 30.0, 0)
    assert segs[0]["end"] == 30.0


def test_fallback_policy():
    assert compression_ratio("abc " * 100) > 2.4
    assert needs_fallback(3.0, -0.2, 0.1) == (True, False)
    assert needs_fallback(1.5, -1.5, 0.1) == (True, True)
    assert needs_fallback(1.5, -1.5, 0.9) == (False, True)           # silence exemption
    assert needs_fallback(1.5, -0.5, 0.9) == (False, True)
    assert should_skip_window(0.9, -1.5) and not should_skip_window(0.9, -0.5)
    assert abs(avg_logprob(-0.5, 9) - (-0.5 * 9 / 10)) < 1e-12
