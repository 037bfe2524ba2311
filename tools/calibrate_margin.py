"""Calibration table of the margin-planted synthetic model's audio bits (vlog_amd/weights.py plant_margin).

The bits are window-level features of the normalised log-mel: projections of the window-mean mel spectrum onto
the leading principal components of the speech-like corpus (vlog_amd.audio.speech_like, clips 0..63), so the
bits are uncorrelated over windows, centred on the corpus median, and scaled by their spread.  Writes
vlog_amd/margin_calib.json (n_mels 80 and 128).  CPU only; a few seconds."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import mel as omel  # noqa: E402  (test infrastructure: the reference log-mel)
from vlog_amd.audio import speech_like  # noqa: E402

N_BITS = 6
W = 64


def main():
    x = np.concatenate([speech_like(30.0, i) for i in range(W)])
    out = {}
    for nm in (80, 128):
        full = omel.log_mel(x, nm)[:, :W * 3000]
        m = full.reshape(nm, W, 3000).mean(-1).T                                     # [W, n_mels]
        c = m - m.mean(0)
        _, _, vt = np.linalg.svd(c, full_matrices=False)
        P = vt[:N_BITS].T                                                            # [n_mels, N_BITS]
        F = m @ P
        out[str(nm)] = {"proj": np.round(P, 6).tolist(), "median": np.round(np.median(F, 0), 6).tolist(),
                        "spread": np.round(F.std(0), 6).tolist(),
                        "frame_std": np.round((full.T @ P).std(0), 6).tolist(),
                        "bit_corr": np.round(np.corrcoef((F > np.median(F, 0)).T), 3).tolist()}
    with open(os.path.join(ROOT, "vlog_amd", "margin_calib.json"), "w") as f:
        json.dump({"corpus": f"speech_like clips 0..{W - 1}, 30 s each", "n_bits": N_BITS, "tables": out}, f)
    print(json.dumps({k: {"spread": v["spread"], "median": v["median"]} for k, v in out.items()}))


if __name__ == "__main__":
    main()
