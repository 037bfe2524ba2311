"""Diagnostic: the decoded size of the margin model's window bits (E[c_j] - E[c'_j] averaged over the 1500 encoder
positions) per window, from the GPU encoder — the quantity the decoder's bit head reads.  Prints per-bit
mean / relative spread of |value| over windows (how exact a magnitude-based reading of the bits could be)."""
import json
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vlog_amd.audio import speech_like  # noqa: E402
from vlog_amd.dims import model_dims  # noqa: E402
from vlog_amd.engine import GpuEngine  # noqa: E402
from vlog_amd.weights import plant_margin, synthetic_state_dict  # noqa: E402

out = {}
for name, W in (("base", 32), ("large-v3", 150)):
    dims = model_dims(name)
    sd = synthetic_state_dict(dims, seed=0)
    plan = plant_margin(sd, dims, 0)
    eng = GpuEngine(dims, sd, 0)
    x = np.concatenate([speech_like(30.0, i) for i in range(W)])
    mel = eng.features(torch.from_numpy(x))
    enc = eng.encode(mel, [3000 * i for i in range(W)], [3000] * W).float()
    c, cr = plan.bit_channels
    v = (enc[:, :, c] - enc[:, :, cr]).mean(1).cpu().numpy()          # [W, n_bits]
    a = np.abs(v)
    out[name] = {"mean_abs": a.mean(0).round(4).tolist(), "rel_std": (a.std(0) / a.mean(0)).round(4).tolist(),
                 "min_abs": a.min(0).round(4).tolist(), "max_abs": a.max(0).round(4).tolist(),
                 "common_scale_rel_std": float((a / a.mean(0)).mean(1).std()),
                 "per_bit_after_common": float(((a / a.mean(0)) / (a / a.mean(0)).mean(1, keepdims=True)).std()),
                 "sign_frac_pos": (v > 0).mean(0).round(3).tolist()}
    print(name, json.dumps(out[name]), flush=True)
    del eng
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/diag_margin_rho.json", "w"))
