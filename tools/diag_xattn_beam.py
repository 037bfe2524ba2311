#!/usr/bin/env python3
"""Diagnostic (builder): tiny beam-5, projected vs factored cross-attention (tests/test_gpu_xattn.py's
beam case), each form's chosen sequence scored by the oracle against the oracle's own beam result.
Prints one JSON line per window."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.decode import GenerateOptions, generate_one, score_sequence  # noqa: E402
from oracle.model import OracleWhisper  # noqa: E402
from tests.test_gpu_xattn import _both, _engine, _sup  # noqa: E402
from vlog_amd.weights import round_bf16  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
    W = 4
    dims, sd, eng, enc = _engine(name, 7, W)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32)
    st = dims.specials
    prompt = [st.sot, st.lang_token("en"), st.transcribe]
    kw = dict(beam_size=5, patience=1.0)

    def run():
        return eng.generate(list(range(W)), [prompt] * W, suppress_tokens=_sup(st), max_length=100, **kw)

    (ra, _), (rb, _) = _both(eng, enc, W, 5 * W, run)
    opt = GenerateOptions(beam_size=5, suppress_tokens=_sup(st), max_length=100)
    encf = enc.float().cpu().numpy()
    for w in range(W):
        cross = orc.cross_kv(encf[w: w + 1])
        r = generate_one(orc, cross, prompt, st, opt)
        out = {"w": w, "same": ra[w].tokens == rb[w].tokens, "oracle_score": r.score,
               "oracle_eq_proj": r.tokens == ra[w].tokens, "oracle_eq_fact": r.tokens == rb[w].tokens}
        for tag, x in (("proj", ra[w]), ("fact", rb[w])):
            ended = len(prompt) + len(x.tokens) < 100
            chosen, best, score = score_sequence(orc, cross, prompt, x.tokens, st, opt, ended)
            out[tag] = {"gpu_score": x.score, "oracle_score_of_seq": score, "finite": bool(np.all(np.isfinite(chosen))),
                        "len": len(x.tokens)}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
