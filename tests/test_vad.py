"""VAD chunking / restore (faster-whisper get_speech_timestamps state machine, collect_chunks,
SpeechTimestampsMap) with crafted speech probabilities — known answers worked out by hand."""
import numpy as np

from vlog_amd.transcribe import Segment, VadOptions, Word
from vlog_amd.vad import SpeechTimestampsMap, collect_chunks, get_speech_timestamps, restore_speech_timestamps

W = 512


def _probs(spec, n_frames):
    p = np.zeros(n_frames)
    for a, b in spec:
        p[a:b] = 0.9
    return p


def test_two_speech_regions_with_long_gap():
    n = 16000 * 20
    frames = -(-n // W)
    p = _probs([(31, 188), (500, 563)], frames)          # ~1.0-6.0 s and ~16.0-18.0 s
    sp = get_speech_timestamps(np.zeros(n, np.float32), VadOptions(), probs=p)
    assert len(sp) == 2
    assert sp[0]["start"] == 31 * W - 6400 and sp[0]["end"] == 188 * W + 6400
    # the second region is followed by < 2 s of silence before EOF, so it is closed at the end of the audio
    assert sp[1]["start"] == 500 * W - 6400 and sp[1]["end"] == n


def test_short_gap_is_bridged():
    n = 16000 * 10
    p = _probs([(10, 60), (90, 140)], -(-n // W))       # gap ~0.96 s < min_silence 2 s -> one chunk
    sp = get_speech_timestamps(np.zeros(n, np.float32), VadOptions(), probs=p)
    assert len(sp) == 1 and sp[0]["start"] == max(0, 10 * W - 6400)


def test_collect_and_restore():
    audio = np.arange(16000 * 10, dtype=np.float32)
    chunks = [{"start": 16000, "end": 32000}, {"start": 80000, "end": 96000}]
    got = collect_chunks(audio, chunks)
    assert got.size == 32000 and got[0] == 16000 and got[16000] == 80000
    m = SpeechTimestampsMap(chunks, 16000)
    assert m.get_original_time(0.5) == 1.5 and m.get_original_time(1.5) == 5.5
    segs = [Segment(1, 0, 0.2, 1.8, " a", [1], -0.1, 1.0, 0.0, None, 0.0),
            Segment(2, 0, 0.4, 1.2, " b", [1], -0.1, 1.0, 0.0,
                    [Word(0.4, 0.9, " x", 0.9), Word(1.1, 1.2, " y", 0.9)], 0.0)]
    out = list(restore_speech_timestamps(iter(segs), chunks, 16000))
    assert (out[0].start, out[0].end) == (1.2, 5.8)
    assert (out[1].start, out[1].end) == (1.4, 5.2) and out[1].words[1].start == 5.1


def test_segment_end_on_chunk_boundary_stays_in_its_chunk():
    """faster-whisper 1.1 `get_chunk_index(..., is_end=True)`: an end exactly at a chunk's last (collected)
    sample maps with that chunk's offset, not the next chunk's (which would add the 3 s silence gap)."""
    chunks = [{"start": 16000, "end": 32000}, {"start": 80000, "end": 96000}]
    m = SpeechTimestampsMap(chunks, 16000)
    assert m.get_original_time(1.0, is_end=True) == 2.0            # end of chunk 0 in collected time
    assert m.get_original_time(1.0) == 5.0                          # a START at that instant belongs to chunk 1
    segs = [Segment(1, 0, 0.2, 1.0, " a", [1], -0.1, 1.0, 0.0, None, 0.0)]
    out = list(restore_speech_timestamps(iter(segs), chunks, 16000))
    assert (out[0].start, out[0].end) == (1.2, 2.0)
