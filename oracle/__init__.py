"""oracle/ — CPU restatement of the reference's Whisper transcription path.  TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import anything from
here, and only as the checker.  The product (`vlog_amd/`) never imports, links or executes this package;
its GPU path fails loudly when the HIP library is missing instead of falling back to a CPU path.

What is restated, and where the semantics come from
---------------------------------------------------
The reference (filthyrake/vlog) contains no arithmetic of its own for this path: the worker calls
`faster_whisper.WhisperModel(WHISPER_MODEL, device="cpu", compute_type=...)` and
`model.transcribe(str(wav), language=lang, task="transcribe", beam_size=5, vad_filter=True)`
(`worker/transcription.py:78-111`).  faster-whisper (`pyproject.toml:24`, `requirements.txt:18`:
"faster-whisper>=1.0.0", unpinned; restated here at its 1.1.x semantics) and CTranslate2 (transitive) are
NOT installed or vendored in this container, so every file below restates their published algorithm and
cites the upstream function it follows ([FW↑] in SURVEY.md).

Pinning (see DESIGN.md "Oracle and parity"):
  * mel.py     — pinned against transformers 5.15.0's WhisperFeatureExtractor numpy path (same filterbank,
                 same STFT), plus faster-whisper's +160-sample padding / global clamp semantics.
  * model.py   — pinned against transformers' WhisperForConditionalGeneration on identical seeded weights.
  * decode.py  — timestamp rules pinned against transformers' WhisperTimeStampLogitsProcessor
                 (`generation/logits_process.py:1909-2049`); beam search restates openai/CTranslate2.
  * align.py   — DTW / median filter pinned against transformers' `_dynamic_time_warping` /
                 `_median_filter` (`models/whisper/generation_whisper.py:43-116`).
  * vtt goldens (tests/golden/vtt_cases.json) come from the reference's own `generate_webvtt`
    (`worker/transcription.py:37-58`), imported in this container with its DB modules stubbed
    (tests/golden/make_vtt_goldens.py).
The reference's own tests pin no transcription result, so end-to-end parity against
faster-whisper itself is "parity unpinned" unless a faster-whisper install is present on the GPU box.
"""
