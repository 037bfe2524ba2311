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
    from vlog_amd.audio import room_tone
    # the W speech clips, then one window of room tone (the variable plant's quiet bit; its log-mel sits at the
    # file's clamp floor, so it is measured inside a speech file)
    x = np.concatenate([speech_like(30.0, i) for i in range(W)])
    xq = np.concatenate([x, room_tone(30.0, 0)])
    out = {}
    for nm in (80, 128):
        full = omel.log_mel(x, nm)[:, :W * 3000]
        full_q = omel.log_mel(xq, nm)
        m = full.reshape(nm, W, 3000).mean(-1).T                                     # [W, n_mels]
        c = m - m.mean(0)
        _, _, vt = np.linalg.svd(c, full_matrices=False)
        P = vt[:N_BITS].T                                                            # [n_mels, N_BITS]
        F = m @ P
        out[str(nm)] = {"proj": np.round(P, 6).tolist(), "median": np.round(np.median(F, 0), 6).tolist(),
                        "spread": np.round(F.std(0), 6).tolist(),
                        "frame_std": np.round((full.T @ P).std(0), 6).tolist(),
                        "bit_corr": np.round(np.corrcoef((F > np.median(F, 0)).T), 3).tolist()}
        # quiet bit (plant margin_var): bit 0's projection with its centre 60 % of the way from the speech median to
        # room tone's value, so speech windows sit >= 2.5 spreads on one side and silence >= 3 on the other
        f_sil = float(full_q[:, W * 3000: W * 3000 + 3000].mean(-1) @ P[:, 0])
        med0 = float(np.median(F, 0)[0])
        out[str(nm)]["quiet"] = {"silence": round(f_sil, 6), "threshold": round(med0 + 0.6 * (f_sil - med0), 6),
                                 "speech_min_max": [round(float(F[:, 0].min()), 6), round(float(F[:, 0].max()), 6)]}
    with open(os.path.join(ROOT, "vlog_amd", "margin_calib.json"), "w") as f:
        json.dump({"corpus": f"speech_like clips 0..{W - 1}, 30 s each", "n_bits": N_BITS, "tables": out}, f)
    print(json.dumps({k: {"spread": v["spread"], "median": v["median"]} for k, v in out.items()}))


if __name__ == "__main__":
    main()
