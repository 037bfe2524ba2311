"""Diagnostic: where config 5's word alignment spends its time.

large-v3 margin model, 150 windows: beam-5 decode (projected cross form, as the product runs beam groups), then
the batched alignment (WhisperModel.find_alignment -> wm_align_batch) timed end to end and per engine kernel class
(the built-in event profiler, enabled around the alignment call only).  Prints one JSON line.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vlog_amd.audio import speech_like  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.tokenizer import Tokenizer  # noqa: E402
from vlog_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "large-v3"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    mode = int(sys.argv[3]) if len(sys.argv) > 3 else 0          # cross form during the alignment
    dims = model_dims(name)
    eng = GpuEngine(dims, synthetic_state_dict(dims, seed=0, plant="margin"), 0)
    tok = Tokenizer(dims, language="en")
    prompt, sup = list(tok.sot_sequence), list(tok.suppressed_tokens([-1]))
    x = np.concatenate([speech_like(30.0, i) for i in range(W)])
    mel = eng.features(torch.from_numpy(x))
    enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W)
    eng.set_option("cross_mode", mode)
    eng.reserve(W, W * 5)
    eng.cross_kv(enc, 0)
    res, _ = eng.generate(list(range(W)), [prompt] * W, beam_size=5, suppress_tokens=sup, max_length=448)
    st = dims.specials
    texts = [[t for t in r.tokens if t < st.eot] for r in res]
    heads = dims.default_alignment_heads()
    out = {"model": name, "windows": W, "cross_mode": mode, "heads": len(heads),
           "text_tokens_mean": float(np.mean([len(t) for t in texts]))}
    for rep in range(2):
        torch.cuda.synchronize()
        if rep == 1:
            eng.profile(True)
        t0 = time.perf_counter()
        eng.align_batch(list(range(W)), prompt, texts, [3000] * W, heads, median_filter_width=7)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if rep == 1:
            eng.profile(False)
            out["profiled_s"] = round(dt, 4)
            out["classes_ms"] = {k: round(v["ms"], 2) for k, v in eng.profile_read().items() if v["launches"]}
        else:
            out["align_s"] = round(dt, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
