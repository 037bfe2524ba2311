#!/usr/bin/env python3
"""Diagnostic (builder): teacher-forced logits at few rows (the small-M decoder path) for the projected and
factored cross-attention forms, with the small-M GEMM on and off, against the f32 oracle.  One JSON line per
configuration."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.model import OracleWhisper  # noqa: E402
from tests.test_gpu_xattn import _engine  # noqa: E402
from vlog_amd.weights import round_bf16  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "tiny"
    W = 4
    dims, sd, eng, enc = _engine(name, 7, W)
    orc = OracleWhisper(round_bf16(sd), dims, np.float32)
    st = dims.specials
    encf = enc.float().cpu().numpy()
    for n_tok, wins in ((4, [1, 3]), (10, [0, 1, 2]), (8, [0, 1, 2, 3])):
        toks = np.array([[st.sot, st.lang_token("en"), st.transcribe] + list(range(700, 700 + n_tok - 3))] * len(wins))
        refs = [orc.decode(toks[i:i + 1], orc.cross_kv(encf[w:w + 1]))[0][0] for i, w in enumerate(wins)]
        out = {}
        for gemv in (1, 0):
            eng.set_option("decode_gemv", gemv)
            for mode in (0, 1):
                eng.set_option("cross_mode", mode)
                eng.reserve(W, 5 * W)
                eng.cross_kv(enc, 0)
                lg = eng.forward(wins, toks)[0].cpu().numpy()
                err = max(float(np.abs(lg[i] - refs[i]).max()) for i in range(len(wins)))
                out[f"gemv{gemv}_mode{mode}"] = err
        print(json.dumps({"rows": n_tok * len(wins), "max_abs_err_vs_oracle": out}))


if __name__ == "__main__":
    main()
