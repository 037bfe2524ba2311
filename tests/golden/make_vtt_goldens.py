"""Generate tests/golden/vtt_cases.json from the REFERENCE's own WebVTT writer.

Imports `worker.transcription` from /root/reference (read-only) with `api.database` and
`api.webhook_service` stubbed (SURVEY.md §8c recipe; those modules need a database driver that is not
installed), then records `format_timestamp` / `generate_webvtt` outputs for the edge cases listed in
SURVEY.md §8a row A15.  Only inputs and outputs are stored; no reference source is copied.

Run: python tests/golden/make_vtt_goldens.py   (needs /root/reference; the committed JSON is what tests use)
"""
import json
import os
import sys
import types

REF = os.environ.get("VLOG_REFERENCE", "/root/reference")


def load_reference_worker():
    sys.path.insert(0, REF)
    os.environ.setdefault("VLOG_TEST_MODE", "1")
    sys.dont_write_bytecode = True
    db = types.ModuleType("api.database")
    db.configure_database = lambda *a, **k: None
    db.database = None
    db.transcriptions = None
    wh = types.ModuleType("api.webhook_service")
    wh.trigger_webhook_event = lambda *a, **k: None
    sys.modules["api.database"] = db
    sys.modules["api.webhook_service"] = wh
    import worker.transcription as wt  # noqa: E402
    return wt


TIMESTAMPS = [0.0, 0.001, 0.0005, 1.0005, 2.0005, 2.5, 9.999, 59.9994, 59.9995, 59.9996, 60.0, 61.04, 599.5,
              3599.9996, 3600.0, 3661.2345, 35999.999, 36000.0, 360000.5, 12.345678, 0.02, 29.98, 30.0]

SEGMENT_SETS = [
    [],
    [{"start": 0.0, "end": 2.5, "text": " Hello world."}, {"start": 2.5, "end": 61.04, "text": " Second  "}],
    [{"start": 0.0, "end": 0.0, "text": ""}],
    [{"start": 1.0005, "end": 2.0005, "text": "  line one\nline two  "}],
    [{"start": 3599.9996, "end": 3661.2345, "text": " ünïcödé — 日本語 "}],
    [{"start": 0.02 * i, "end": 0.02 * i + 1.37, "text": f" seg {i}"} for i in range(0, 1500, 137)],
    [{"start": 360000.5, "end": 360001.25, "text": " long file"}],
]


def main():
    wt = load_reference_worker()
    out = {
        "source": "worker/transcription.py:37-58 (filthyrake/vlog @ 2026-01-16), format_timestamp + generate_webvtt",
        "format_timestamp": [[t, wt.format_timestamp(t)] for t in TIMESTAMPS],
        "generate_webvtt": [[segs, wt.generate_webvtt(segs)] for segs in SEGMENT_SETS],
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vtt_cases.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
