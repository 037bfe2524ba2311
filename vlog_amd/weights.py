"""Model weights: local HF-format directories and seeded synthetic weights.

The reference passes a model *name* (`WHISPER_MODEL`, `config.py:263`) that faster-whisper resolves by
downloading from the HF Hub (`worker/transcription.py:81-85`).  This engine never downloads anything:
`resolve_model()` maps

  * a local directory with `config.json` + `model.safetensors` (HF Whisper layout) -> those weights;
  * a local CTranslate2 directory (`model.bin`, the layout a faster-whisper deployment uses) -> its weights,
    dequantised to float32 (vlog_amd/ct2.py);
  * a name with `VLOG_AMD_MODEL_DIR_<name>` (or `VLOG_AMD_MODEL_ROOT/<name>`) set -> that directory;
  * `"synthetic:<name>[:seed][:margin]"` -> random-init weights of that architecture (there are no real
    checkpoints in this environment; BASELINE.md "Synthetic audio"); `:margin` adds the decisive planted
    decoder program (plant_margin) used for the token-identity / WER / timestamp gates;

and raises a ValueError otherwise.

Synthetic init follows the upstream initialiser shape (normal(0, 0.02) for linear/conv/embedding weights,
sinusoids for the encoder positions) but gives biases and LayerNorm affines small random values so every
bias/affine path is exercised.  `eot_after` optionally plants one direction in the decoder positional
embedding and the <|endoftext|> embedding row so that greedy decoding ends after a speech-like number of
tokens instead of running to the 448-token limit (documented in DESIGN.md; both engines see identical
weights, so parity is unaffected).
"""
from __future__ import annotations

import hashlib
import json
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .dims import ModelDims, custom_dims, model_dims


def _gen(seed: int, name: str) -> torch.Generator:
    h = int.from_bytes(hashlib.sha256(f"{seed}:{name}".encode()).digest()[:8], "little") & ((1 << 63) - 1)
    g = torch.Generator(device="cpu")
    g.manual_seed(h)
    return g


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> torch.Tensor:
    inc = np.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-inc * torch.arange(channels // 2, dtype=torch.float64))
    t = torch.arange(length, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([torch.sin(t), torch.cos(t)], dim=1).float()


def weight_shapes(dims: ModelDims) -> Dict[str, Tuple[int, ...]]:
    d, f, m = dims.n_state, dims.n_ffn, dims.n_mels
    s: Dict[str, Tuple[int, ...]] = {
        "model.encoder.conv1.weight": (d, m, 3), "model.encoder.conv1.bias": (d,),
        "model.encoder.conv2.weight": (d, d, 3), "model.encoder.conv2.bias": (d,),
        "model.encoder.embed_positions.weight": (dims.n_audio_ctx, d),
        "model.encoder.layer_norm.weight": (d,), "model.encoder.layer_norm.bias": (d,),
        "model.decoder.embed_tokens.weight": (dims.n_vocab, d),
        "model.decoder.embed_positions.weight": (dims.n_text_ctx, d),
        "model.decoder.layer_norm.weight": (d,), "model.decoder.layer_norm.bias": (d,),
    }

    def attn(p):
        s.update({p + "q_proj.weight": (d, d), p + "q_proj.bias": (d,), p + "k_proj.weight": (d, d),
                  p + "v_proj.weight": (d, d), p + "v_proj.bias": (d,), p + "out_proj.weight": (d, d),
                  p + "out_proj.bias": (d,)})

    def ln(p):
        s.update({p + "weight": (d,), p + "bias": (d,)})

    def mlp(p):
        s.update({p + "fc1.weight": (f, d), p + "fc1.bias": (f,), p + "fc2.weight": (d, f), p + "fc2.bias": (d,)})

    for i in range(dims.n_enc_layer):
        p = f"model.encoder.layers.{i}."
        attn(p + "self_attn."); ln(p + "self_attn_layer_norm."); ln(p + "final_layer_norm."); mlp(p)
    for i in range(dims.n_dec_layer):
        p = f"model.decoder.layers.{i}."
        attn(p + "self_attn."); ln(p + "self_attn_layer_norm."); attn(p + "encoder_attn.")
        ln(p + "encoder_attn_layer_norm."); ln(p + "final_layer_norm."); mlp(p)
    return s


def synthetic_state_dict(dims: ModelDims, seed: int = 0, eot_after: Optional[int] = None,
                         std: float = 0.02, plant: Optional[str] = None) -> Dict[str, torch.Tensor]:
    """Seeded random-init weights (float32, CPU), HF naming.  Per-tensor generators make any subset
    reproducible on its own.  plant="margin": the decisive planted program of plant_margin (eot_after is
    ignored: the script ends the window)."""
    sd: Dict[str, torch.Tensor] = {}
    for name, shape in weight_shapes(dims).items():
        g = _gen(seed, name)
        if name == "model.encoder.embed_positions.weight":
            t = sinusoids(shape[0], shape[1])
        elif name.endswith("layer_norm.weight"):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name.endswith(".bias"):
            t = std * torch.randn(shape, generator=g)
        else:
            t = std * torch.randn(shape, generator=g)
        sd[name] = t.float()
    if plant in ("margin", "margin_var"):
        plant_margin(sd, dims, seed, variable=plant == "margin_var")
    elif plant is not None:
        raise ValueError(f"unknown plant {plant!r}")
    elif eot_after is not None:
        plant_eot(sd, dims, eot_after, seed)
    return sd


# Final decoder residual-stream std of the seeded random init, by decoder depth (measured with the oracle on
# teacher-forced sequences; used to scale the planted <|endoftext|> ramp to the model's depth).
_RESID_STD = {4: 0.41, 6: 0.67, 12: 1.50, 24: 2.94, 32: 4.5}


def _resid_std(n_layers: int) -> float:
    ks = sorted(_RESID_STD)
    if n_layers in _RESID_STD:
        return _RESID_STD[n_layers]
    lo = max([k for k in ks if k <= n_layers], default=ks[0])
    hi = min([k for k in ks if k >= n_layers], default=ks[-1])
    if lo == hi:
        return _RESID_STD[lo] * n_layers / lo
    t = (n_layers - lo) / (hi - lo)
    return _RESID_STD[lo] * (1 - t) + _RESID_STD[hi] * t


EOT_KAPPA = 4.0


def plant_eot(sd: Dict[str, torch.Tensor], dims: ModelDims, eot_after: int, seed: int = 0) -> None:
    """Plant one direction u: E[<|endoftext|>] = c_e * u (the norm of a random row) and decoder position p
    carries slope * p * u with slope = EOT_KAPPA * s_L / (c_e * eot_after) (s_L = final residual std for this
    decoder depth), so the <|endoftext|> logit rises by about EOT_KAPPA over `eot_after` positions and
    greedy decoding ends near there."""
    d = dims.n_state
    g = _gen(seed, "plant_eot")
    u = torch.randn(d, generator=g)
    u = u / u.norm()
    pos = sd["model.decoder.embed_positions.weight"]
    c_e = 0.02 * float(np.sqrt(d))            # same norm as any random embedding row
    slope = EOT_KAPPA * _resid_std(dims.n_dec_layer) / (c_e * float(eot_after))
    pos += slope * torch.arange(pos.shape[0], dtype=torch.float32)[:, None] * u[None, :]
    sd["model.decoder.embed_tokens.weight"][dims.specials.eot] = c_e * u


# ----------------------------------------------------------------------------- margin-planted synthetic model
# The audio bits: window-level features of the normalised log-mel (projections of the window-mean spectrum onto
# the corpus' leading principal components, so the bits are uncorrelated over windows), centred on the corpus
# median.  vlog_amd/margin_calib.json, written by tools/calibrate_margin.py; only the centring and scale of the
# bits depend on it.
N_BITS = 6


def _margin_calib(n_mels: int) -> dict:
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "margin_calib.json")) as f:
        t = json.load(f)["tables"]
    if str(n_mels) not in t:
        raise ValueError(f"no margin-model calibration for n_mels={n_mels}")
    return t[str(n_mels)]


@dataclass
class MarginPlan:
    """The planted decoder program.  slots[k] = tokens of script slot k (one token, or a +/- pair chosen by
    bits[k]); kinds[k] in {"text", "ts", "ts_final"}."""
    slots: List[Tuple[int, ...]]
    kinds: List[str]
    bits: List[Optional[int]]
    first_key: Tuple[int, ...]          # prompt tokens whose unit emits slot 0 (the first timestamp)
    # encoder output channels carrying the window bits (bit j = E[c_ch[j]] - E[c_ref[j]]), set by plant_margin
    bit_channels: Optional[Tuple[List[int], List[int]]] = None
    # variable-length script (plant "margin_var"): (slot k of a timestamp, threshold T) — the window ends with
    # <|endoftext|> right after that timestamp when its level L = sum_j LEVEL_W[j] * bit_j exceeds T (first such k)
    exits: List[Tuple[int, int]] = field(default_factory=list)
    # variable plant: the sign the quiet bit carries for a silent window (bit_channels[.][7])
    quiet_sign: int = 0


# Variable-length script (plant "margin_var"): 16 segments (up to ~225 tokens), level weights of the six bits (bit 0,
# the corpus' first principal component = the window's mean log-mel energy, i.e. how much of it is speech, weighs
# 3 and with a negative sign: more speech -> a lower level -> a later exit), and the exits: (segment whose end
# timestamp may end the window (-1: the first timestamp), threshold).  Levels L in {-8, ..., 8} step 2 follow a
# shifted binomial; thresholds sit at odd values, so every decision has a full level of margin:
#   L = 8 -> 1 token, 6 -> 5 (the 3-token first segment), 4 -> ~48, 2 -> ~77, 0 -> ~92, -2 -> ~121, -4 -> ~150,
#   -6 -> ~179, -8 -> the whole script (~222); mean ~97 over the level distribution.
VAR_SEGMENTS = 16
LEVEL_W = (-3, 1, 1, 1, 1, 1)
# the quiet bit's weight in the first exit's test (QUIET_W - 7 > 0 for a silent window, -QUIET_W - 7 < 0 for speech)
# and the slope of its encoder clip
QUIET_W = 14
K_Q = 2.0


def level_weights(n_mels: int) -> Tuple[int, ...]:
    """LEVEL_W with bit 0's sign oriented so that MORE speech lowers the level (a later exit): the first principal
    component's sign is arbitrary per calibration table (n_mels 80: it grows with the window's energy, 128: it
    falls), so the weight follows the sign of its loadings."""
    p0 = float(np.sum(np.asarray(_margin_calib(n_mels)["proj"])[:, 0]))
    return (LEVEL_W[0] * (1 if p0 >= 0 else -1),) + tuple(LEVEL_W[1:])
VAR_EXITS = ((-1, 7), (0, 5), (3, 3), (5, 1), (6, -1), (8, -3), (10, -5), (12, -7))


def margin_plan(dims: ModelDims, seed: int = 0, n_segments: int = 8, variable: bool = False) -> MarginPlan:
    st = dims.specials
    if variable:
        n_segments = VAR_SEGMENTS
    rng = np.random.default_rng(int.from_bytes(hashlib.sha256(f"{seed}:margin_plan".encode()).digest()[:8], "little"))
    text_ids = rng.choice(np.arange(1000, st.eot - 1000), size=400 if not variable else 800, replace=False).tolist()
    slots: List[Tuple[int, ...]] = [(st.timestamp_begin,)]
    kinds, bits = ["ts"], [None]
    span = 28.0 / n_segments
    bit = 0
    for m in range(n_segments):
        n = int(rng.integers(10, 15))
        branch_at = set(rng.choice(np.arange(1, n - 1), size=2, replace=False).tolist())
        if variable and m == 0:
            n, branch_at = 3, set()                      # a short first segment: the 5-token exit
        for j in range(n):
            if j in branch_at and j - 1 not in branch_at:
                slots.append((text_ids.pop(), text_ids.pop()))
                bits.append(bit % N_BITS)
                bit += 1
            else:
                slots.append((text_ids.pop(),))
                bits.append(None)
            kinds.append("text")
        a = int(round((m + 1) * span / 0.02))
        if m == n_segments - 1:
            slots.append((st.timestamp_begin + a,))
            kinds.append("ts_final")
            bits.append(None)
        elif m % 2 == 1 and not variable:                # a segment boundary that moves with the audio
            slots.append((st.timestamp_begin + a, st.timestamp_begin + a + 8))
            kinds.append("ts")
            bits.append(bit % N_BITS)
            bit += 1
        else:
            slots.append((st.timestamp_begin + a,))
            kinds.append("ts")
            bits.append(None)
    first_key = (st.transcribe,) if dims.multilingual else (st.sot,)
    plan = MarginPlan(slots, kinds, bits, first_key)
    if variable:
        ends = [k for k, kd in enumerate(kinds) if kd in ("ts", "ts_final") and k > 0]     # segment m ends at ends[m]
        plan.exits = [(0 if m < 0 else ends[m], t) for m, t in VAR_EXITS]
    return plan


def plant_margin(sd: Dict[str, torch.Tensor], dims: ModelDims, seed: int = 0, variable: bool = False) -> MarginPlan:
    """Plant a decisive, audio-dependent decoder program into seeded random weights (test model for the
    north_star token-identity / WER / timestamp gates).

    Random-init Whisper weights give near-tied logits (top-1 vs top-2 and the timestamp-forcing gap sit within
    bf16 noise), so token identity between two correct implementations is a coin toss.  A trained model is
    decisive; this plants that property while keeping every random weight elsewhere:

    * decoder layer 0's MLP holds a successor table: hidden unit k fires on script slot k's token direction
      (fc1 row = that direction, bias = threshold) and writes the next slot's direction (fc2 column), so the
      next token wins by thousands of nats over the input token and every random contribution;
    * timestamps: a timestamp slot's unit writes both its own direction (the repeated timestamp of a pair;
      the rules mask text after the first) and the next text slot's (the rules mask timestamps after the
      second); the last one writes <|endoftext|>;
    * audio dependence: N_BITS window-level bits.  The conv stem computes mel-bin projections (centred on the
      corpus median); one uniform-attention head of encoder layer 0 averages them over the window into
      channels no other layer writes, so the encoder output carries each window's bit value with an exact sign
      in bf16 and in fp8; one uniform head of decoder layer 0's cross-attention reads them and writes them along
      a bit direction; a branch slot's two tokens differ by +-alpha times that direction, so the bit's sign
      picks the token (and segment boundaries move with it).
    The encoder channel trick: bit channel m and its reference m' receive identical (zero) writes from every
    random layer and share LayerNorm affines, so E[m] - E[m'] is the planted value alone.

    variable=True (plant "margin_var", margin_plan VAR_*): a 16-segment script whose length follows the audio.  A
    seventh, constant bit (+1 for every window) rides the same channels and head, so every bit the decoder reads is
    s_j * rho_w with ONE common per-window scale rho_w; the window's level L = sum_j LEVEL_W[j] s_j is compared with a
    threshold T as rho_w (L - T), whose sign is exact.  At each exit timestamp k, two units of decoder layer 2's MLP
    key on that position (the repeat + next-text directions the successor table writes there) and differ only by
    the level term: A = GELU(P + g (L - T) rho_w), B = GELU(P); A - B writes <|endoftext|>, so the window ends
    after timestamp k iff L > T (GELU is monotonic where B sits), by a margin of one level (thousands of nats at
    large-v3); elsewhere both units are off."""
    d, H = dims.n_state, dims.n_head
    hd = d // H
    st = dims.specials
    plan = margin_plan(dims, seed, variable=variable)
    g = _gen(seed, "plant_margin")
    rng = np.random.default_rng(int.from_bytes(hashlib.sha256(f"{seed}:plant_margin".encode()).digest()[:8], "little"))

    # ---- encoder: stem bit features, averaging head, protected channels
    nb = N_BITS
    ch = rng.choice(d, size=6 * nb, replace=False)
    s_ch, s_ref, m_ch, m_ref, c_ch, c_ref = (ch[i * nb:(i + 1) * nb] for i in range(6))
    k_ch = k_ref = None
    qch = None
    if variable:
        rng_v = np.random.default_rng(int.from_bytes(hashlib.sha256(f"{seed}:plant_margin_var".encode()).digest()[:8], "little"))
        k_ch, k_ref = (int(c) for c in rng_v.choice(np.setdiff1d(np.arange(d), ch), size=2, replace=False))
        # the quiet bit's six channels (stem, its reference, window mean, its reference, carrier, its reference),
        # drawn after the constant bit's two
        qch = [int(c) for c in rng_v.choice(np.setdiff1d(np.arange(d), np.concatenate([ch, [k_ch, k_ref]])), size=6,
                                            replace=False)]
    cal = _margin_calib(dims.n_mels)
    P = torch.tensor(cal["proj"], dtype=torch.float32)               # [n_mels, nb]
    med, fstd = cal["median"], cal["frame_std"]
    g1 = [0.25 / f for f in fstd]                                    # 4 frame-sigma -> GELU argument +-1 around b1
    spread = [g * sp for g, sp in zip(g1, cal["spread"])]
    b1 = 3.0
    c1w, c1b = sd["model.encoder.conv1.weight"], sd["model.encoder.conv1.bias"]       # [d, n_mels, 3]
    c2w, c2b = sd["model.encoder.conv2.weight"], sd["model.encoder.conv2.bias"]       # [d, d, 3]
    gelu_b1 = float(0.5 * b1 * (1.0 + math.erf(b1 / math.sqrt(2.0))))
    if variable:                                         # the constant and quiet bits' channels: no stem writes
        for c in [k_ch, k_ref] + qch:
            c1w[c] = 0.0; c1b[c] = 0.0; c2w[c] = 0.0; c2b[c] = 0.0
        # quiet bit: bit 0's projection centred at the calibrated quiet threshold (between speech and room tone)
        # instead of the corpus median, so its sign says "this window is silence"
        qs, qs_ref = qch[0], qch[1]
        thr_q = float(cal["quiet"]["threshold"])
        c1w[qs, :, 1] = g1[0] * P[:, 0]
        c1b[qs] = b1 - g1[0] * thr_q
        c1b[qs_ref] = b1
        c2w[qs, qs, 1] = 1.0
        c2w[qs_ref, qs_ref, 1] = 1.0
        c2b[qs] = b1 - gelu_b1
        c2b[qs_ref] = b1 - gelu_b1
    for j in range(nb):
        for c in (s_ch[j], s_ref[j], m_ch[j], m_ref[j], c_ch[j], c_ref[j]):
            c1w[c] = 0.0; c1b[c] = 0.0; c2w[c] = 0.0; c2b[c] = 0.0
        c1w[s_ch[j], :, 1] = g1[j] * P[:, j]
        c1b[s_ch[j]] = b1 - g1[j] * float(med[j])
        c1b[s_ref[j]] = b1
        c2w[s_ch[j], s_ch[j], 1] = 1.0                   # GELU(y + b1) - GELU(b1) + b1 through the second GELU
        c2w[s_ref[j], s_ref[j], 1] = 1.0
        c2b[s_ch[j]] = b1 - gelu_b1
        c2b[s_ref[j]] = b1 - gelu_b1
    pos = sd["model.encoder.embed_positions.weight"]
    pos[:, torch.as_tensor(ch)] = 0.0
    if variable:
        pos[:, [k_ch, k_ref] + qch] = 0.0
    # layer 0, head h_e: uniform attention (q = 0) averaging (LN[s] - LN[s']) into channel m
    h_e = 0
    p0 = "model.encoder.layers.0.self_attn."
    sl = slice(h_e * hd, (h_e + 1) * hd)
    sd[p0 + "q_proj.weight"][sl] = 0.0
    sd[p0 + "q_proj.bias"][sl] = 0.0
    sd[p0 + "v_proj.weight"][sl] = 0.0
    sd[p0 + "v_proj.bias"][sl] = 0.0
    sd[p0 + "out_proj.weight"][:, sl] = 0.0
    s_enc = _resid_std(dims.n_enc_layer)
    for j in range(nb):
        sd[p0 + "v_proj.weight"][h_e * hd + j, s_ch[j]] = 1.0
        sd[p0 + "v_proj.weight"][h_e * hd + j, s_ref[j]] = -1.0
    if variable:                                         # the quiet bit's window mean: head dimension nb
        sd[p0 + "v_proj.weight"][h_e * hd + nb, qch[0]] = 1.0
        sd[p0 + "v_proj.weight"][h_e * hd + nb, qch[1]] = -1.0
    # the layer-0 LayerNorm affines of s and s' equal, so LN[s] - LN[s'] is the stem difference / sigma_t alone
    ln0w, ln0b = sd["model.encoder.layers.0.self_attn_layer_norm.weight"], sd["model.encoder.layers.0.self_attn_layer_norm.bias"]
    ln0w[torch.as_tensor(s_ref)] = ln0w[torch.as_tensor(s_ch)]
    ln0b[torch.as_tensor(s_ref)] = ln0b[torch.as_tensor(s_ch)]
    if variable:
        ln0w[qch[1]] = ln0w[qch[0]]
        ln0b[qch[1]] = ln0b[qch[0]]
    prot = torch.as_tensor(np.concatenate([m_ch, m_ref, c_ch, c_ref] + ([[k_ch, k_ref], qch[2:]] if variable else [])))
    for i in range(dims.n_enc_layer):
        p = f"model.encoder.layers.{i}."
        for w in ("self_attn.out_proj", "fc2"):
            sd[p + w + ".weight"][prot] = 0.0
            sd[p + w + ".bias"][prot] = 0.0
    for j in range(nb):
        # window-mean of (LN[s] - LN[s']) has spread ~ spread_j / 0.72 (layer-0 LN std: the sinusoid table)
        sd[p0 + "out_proj.weight"][m_ch[j], h_e * hd + j] = float(s_enc * 0.72 / spread[j])
    if variable:
        sd[p0 + "out_proj.weight"][qch[2], h_e * hd + nb] = float(s_enc * 0.72 / spread[0])

    def same_affine(ln: str, a, b):
        w_, b_ = sd[ln + ".weight"], sd[ln + ".bias"]
        w_[torch.as_tensor(b)] = w_[torch.as_tensor(a)]
        b_[torch.as_tensor(b)] = b_[torch.as_tensor(a)]

    # layer-0 MLP: a saturating clip of each window bit into channel c (two GELU units per bit:
    # o/2s * (GELU(s(Ky + 1)) - GELU(s(Ky - 1))) - o/2 = clip(Ky, -1, 1) * o/2 with the zero exactly at y = 0,
    # since GELU(x) - GELU(-x) = x), so all but a sliver of windows carry a full-size bit
    same_affine("model.encoder.layers.0.final_layer_norm", m_ch, m_ref)
    if variable:
        same_affine("model.encoder.layers.0.final_layer_norm", [qch[2]], [qch[3]])
    pf = "model.encoder.layers.0."
    f1w, f1b, f2w, f2b = (sd[pf + n] for n in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"))
    # the variable-length plant reads the bits' signs as a level too: a 20x steeper clip leaves a 20x thinner sliver
    # of windows with a partly saturated bit
    s_g, K, o_half = 8.0, (1000.0 if variable else 50.0), s_enc
    for j in range(nb):
        for u, sgn in ((2 * j, 1.0), (2 * j + 1, -1.0)):
            f1w[u] = 0.0
            f1w[u, m_ch[j]] = s_g * K
            f1w[u, m_ref[j]] = -s_g * K
            f1b[u] = sgn * s_g
            f2w[:, u] = 0.0
        f2w[c_ch[j], 2 * j] = o_half / s_g
        f2w[c_ch[j], 2 * j + 1] = -o_half / s_g
        f2b[c_ch[j]] = -o_half
    same_affine("model.encoder.layer_norm", c_ch, c_ref)
    if variable:
        # the constant bit: two units with fixed pre-activations s(2 + 1), s(2 - 1) (clip(2) = +1 exactly), and every
        # carrying channel with a unit final-LayerNorm affine, so all seven bits leave the encoder as s_j * rho_w
        # with one common per-window scale rho_w = o_half * mean_t rstd_t
        for u, b in ((2 * nb, 3.0 * s_g), (2 * nb + 1, 1.0 * s_g)):
            f1w[u] = 0.0
            f1b[u] = b
            f2w[:, u] = 0.0
        f2w[k_ch, 2 * nb] = o_half / s_g
        f2w[k_ch, 2 * nb + 1] = -o_half / s_g
        f2b[k_ch] = -o_half
        # the quiet bit: the saturating clip of its window mean into its carrier, with a gentle slope K_Q: every
        # window sits >= 2.5 spreads from the quiet threshold, so it saturates all the same, and its GELU units stay
        # below 256 where bf16 resolves their difference (the data bits' K = 1000 units reach ~1e5, where bf16 keeps
        # nothing of the 2 s_g difference: deterministic, but not the designed magnitude, on a window whose positions
        # are all alike, as room tone's are)
        qm, qm_ref, qc, qc_ref = qch[2:]
        for u, sgn in ((2 * nb + 2, 1.0), (2 * nb + 3, -1.0)):
            f1w[u] = 0.0
            f1w[u, qm] = s_g * K_Q
            f1w[u, qm_ref] = -s_g * K_Q
            f1b[u] = sgn * s_g
            f2w[:, u] = 0.0
        f2w[qc, 2 * nb + 2] = o_half / s_g
        f2w[qc, 2 * nb + 3] = -o_half / s_g
        f2b[qc] = -o_half
        lnw, lnb = sd["model.encoder.layer_norm.weight"], sd["model.encoder.layer_norm.bias"]
        carry = torch.as_tensor(np.concatenate([c_ch, c_ref, [k_ch, k_ref, qc, qc_ref]]))
        lnw[carry] = 1.0
        lnb[carry] = 0.0

    # ---- decoder: orthonormal directions
    slot_dirs = len(plan.slots)
    n_dirs = slot_dirs + nb + 4 + (2 if variable else 0)
    q, _ = torch.linalg.qr(torch.randn(d, n_dirs, generator=g, dtype=torch.float64))
    V = q.T.float()                                      # rows: unit, mutually orthogonal
    v_slot = V[:slot_dirs]
    v_bit = V[slot_dirs: slot_dirs + nb]
    v_sot, v_en, v_eot, v_task = V[slot_dirs + nb: slot_dirs + nb + 4]
    v_const = V[slot_dirs + nb + 4] if variable else None
    v_quiet = V[slot_dirs + nb + 5] if variable else None
    N = _resid_std(dims.n_dec_layer) * math.sqrt(d)     # norm of the random residual at the final LayerNorm
    R = 6.0 * N                                         # planted token embedding norm
    Bn = 5.0 * R                                        # successor write (> alpha * the largest bit term)
    alpha = 0.5
    E = sd["model.decoder.embed_tokens.weight"]
    for k, toks in enumerate(plan.slots):
        if len(toks) == 1:
            E[toks[0]] = R * v_slot[k]
        else:
            b = v_bit[plan.bits[k]]
            E[toks[0]] = R * (v_slot[k] + alpha * b) / math.sqrt(1 + alpha ** 2)
            E[toks[1]] = R * (v_slot[k] - alpha * b) / math.sqrt(1 + alpha ** 2)
    E[st.eot] = R * v_eot
    E[st.sot] = R * v_sot
    if dims.multilingual:
        E[st.lang_token("en")] = R * v_en
        E[st.transcribe] = R * v_task
    # cross-attention head h_d of layer 1 (after the successor table, so the table's keys never see the bit
    # terms): uniform attention reading E[m] - E[m'] into the bit directions
    h_d = 0
    pc = f"model.decoder.layers.{min(1, dims.n_dec_layer - 1)}.encoder_attn."
    sl = slice(h_d * hd, (h_d + 1) * hd)
    sd[pc + "q_proj.weight"][sl] = 0.0
    sd[pc + "q_proj.bias"][sl] = 0.0
    sd[pc + "v_proj.weight"][sl] = 0.0
    sd[pc + "v_proj.bias"][sl] = 0.0
    sd[pc + "out_proj.weight"][:, sl] = 0.0
    S_d = 2.0 * R            # saturated window bits E[c] - E[c'] ~ +-1 -> +-2R along the bit direction
    for j in range(nb):
        sd[pc + "v_proj.weight"][h_d * hd + j, c_ch[j]] = 1.0
        sd[pc + "v_proj.weight"][h_d * hd + j, c_ref[j]] = -1.0
        sd[pc + "out_proj.weight"][:, h_d * hd + j] = S_d * v_bit[j]
    if variable:
        sd[pc + "v_proj.weight"][h_d * hd + nb, k_ch] = 1.0
        sd[pc + "v_proj.weight"][h_d * hd + nb, k_ref] = -1.0
        sd[pc + "out_proj.weight"][:, h_d * hd + nb] = S_d * v_const
        sd[pc + "v_proj.weight"][h_d * hd + nb + 1, qch[4]] = 1.0
        sd[pc + "v_proj.weight"][h_d * hd + nb + 1, qch[5]] = -1.0
        sd[pc + "out_proj.weight"][:, h_d * hd + nb + 1] = S_d * v_quiet
    # layer-0 MLP successor table
    pm = "model.decoder.layers.0."
    fc1w, fc1b = sd[pm + "fc1.weight"], sd[pm + "fc1.bias"]
    fc2w = sd[pm + "fc2.weight"]
    sq = math.sqrt(d)
    gam, theta = 1.0, 0.3 * math.sqrt(d)
    a_ref = gam * sq * 0.85 - theta                     # activation at a typical match (cos ~ 0.85)
    units = []                                          # (key direction, write direction)
    for k in range(len(plan.slots) - 1):
        nxt = v_slot[k + 1]
        if plan.kinds[k] == "ts":
            units.append((v_slot[k], v_slot[k] + nxt))  # repeat (pair) + next text slot
        else:
            units.append((v_slot[k], nxt))
    units.append((v_slot[-1], v_eot))                   # the last timestamp -> <|endoftext|>
    if dims.multilingual:
        units.append((v_task, v_slot[0]))
        units.append((v_sot, v_en))                     # language detection / no-speech position
    else:
        units.append((v_sot, v_slot[0]))
    for u, (key, write) in enumerate(units):
        fc1w[u] = gam * key
        fc1b[u] = -theta
        fc2w[:, u] = Bn * write / a_ref
    if variable:
        # Exits, in two stages (decoder layers 2 and 3; unit LayerNorm affines there so the keys read undistorted).
        # Layer 2: per exit e, the window's level test as a saturated clip into its own direction,
        #   I_e = +-o_I (sign of rho_w (L - T_e), exact: the threshold rides the constant bit),
        # the same at every position; it also writes a ballast M along v_ball, which layer 3's fc2 bias removes, so
        # layer 3's LayerNorm sees |x| ~ M at every position whatever the bit magnitudes (the position keys below are
        # then calibrated for every model width).  Layer 3: per exit two units keyed on the exit position (the
        # repeat + next-text directions the successor table writes after timestamp k: cos ~ 0.37 there, <= 0.17
        # elsewhere) that differ only by +-gamma I_e: A - B writes +-Bx gamma o_I of <|endoftext|>, ending the window
        # after timestamp k iff L > T_e (12 R of <|endoftext|> against the repeat's 6 R), bounded either way.
        assert dims.n_dec_layer >= 4, "the variable-length plant needs >= 4 decoder layers"
        n_ex = len(plan.exits)
        qx, _ = torch.linalg.qr(torch.cat([V.T.double(), torch.randn(d, n_ex + 1, generator=g, dtype=torch.float64)], 1))
        Vx = qx.T[V.shape[0]:].float()                  # orthogonal to every planted direction
        v_ind, v_ball = Vx[:n_ex], Vx[n_ex]
        lw = level_weights(dims.n_mels)
        lev = sum(lw[j] * v_bit[j] for j in range(nb))
        scale = 35.8 / sq                               # pre-activations in the large-v3 scale for every width
        o_I, M = 2.0 * R, 20.0 * R
        p2, p3 = "model.decoder.layers.2.", "model.decoder.layers.3."
        for pl in (p2, p3):
            sd[pl + "final_layer_norm.weight"][:] = 1.0
            sd[pl + "final_layer_norm.bias"][:] = 0.0
        f1a, b1a, f2a, b2a = (sd[p2 + n] for n in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"))
        s_c, K_c = 8.0, 5.0 * scale
        # the first exit (one token: the window ends after its first timestamp) reads the quiet bit alone:
        # QUIET_W q_s - T, q_s = +1 for a silent window, so every silent window ends there and no speech window does
        q_sign = 1.0 if float(cal["quiet"]["silence"]) > thr_q else -1.0
        for e, (k, T) in enumerate(plan.exits):
            test = QUIET_W * q_sign * v_quiet - T * v_const if e == 0 else lev - T * v_const
            for u, sgn in ((2 * e, 1.0), (2 * e + 1, -1.0)):
                f1a[u] = s_c * K_c * test
                b1a[u] = sgn * s_c
                f2a[:, u] = sgn * (o_I / s_c) * v_ind[e]
            b2a -= o_I * v_ind[e]
        b2a += M * v_ball
        f1b3, b1b3, f2b3, b2b3 = (sd[p3 + n] for n in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"))
        beta, gam_x, delta = 10.0 * scale, 5.0 * scale, 40.0
        th = beta * sq * 7.78 / 21.0 - delta            # B sits DELTA above zero at the exit position
        Bx = 0.7 * R
        for e, (k, T) in enumerate(plan.exits):
            assert plan.kinds[k] == "ts" and len(plan.slots[k]) == 1 and len(plan.slots[k + 1]) == 1
            u_k = (v_slot[k] + v_slot[k + 1]) / math.sqrt(2.0)
            ua, ub = 2 * e, 2 * e + 1
            f1b3[ua] = beta * u_k + gam_x * v_ind[e]
            f1b3[ub] = beta * u_k
            b1b3[ua] = -th
            b1b3[ub] = -th
            f2b3[:, ua] = Bx * v_eot
            f2b3[:, ub] = -Bx * v_eot
        b2b3 -= M * v_ball
    plan.bit_channels = ([int(c) for c in c_ch] + ([k_ch, qch[4]] if variable else []),
                         [int(c) for c in c_ref] + ([k_ref, qch[5]] if variable else []))
    if variable:
        plan.quiet_sign = 1 if float(cal["quiet"]["silence"]) > float(cal["quiet"]["threshold"]) else -1
    return plan


def stored_as_bf16(name: str, t: torch.Tensor) -> bool:
    """Which tensors the engine keeps in bf16: weight matrices and conv kernels.  Biases, LayerNorm affines
    and the position tables stay float32 (vlog_amd/engine.py pack_weights)."""
    return name.endswith(".weight") and t.dim() >= 2 and "embed_positions" not in name


def round_bf16(sd: Dict[str, torch.Tensor]) -> Dict[str, np.ndarray]:
    """The values the GPU engine actually stores, as float32 numpy arrays for the oracle."""
    return {k: (v.to(torch.bfloat16).float() if stored_as_bf16(k, v) else v.float()).numpy() for k, v in sd.items()}


# ----------------------------------------------------------------------------- local model directories
def dims_from_hf_config(cfg: dict, name: str = "local") -> ModelDims:
    heads = ()
    if cfg.get("alignment_heads"):
        heads = tuple(tuple(x) for x in cfg["alignment_heads"])
    return custom_dims(name, cfg["num_mel_bins"], cfg["d_model"], cfg["encoder_attention_heads"],
                       cfg["encoder_layers"], cfg["decoder_layers"], cfg["vocab_size"],
                       cfg["vocab_size"] >= 51865, alignment_heads=heads)


def load_hf_dir(path: str) -> Tuple[ModelDims, Dict[str, torch.Tensor]]:
    from safetensors.torch import load_file

    with open(os.path.join(path, "config.json")) as f:
        cfg = json.load(f)
    dims = dims_from_hf_config(cfg, os.path.basename(os.path.normpath(path)))
    sd: Dict[str, torch.Tensor] = {}
    for fn in sorted(os.listdir(path)):
        if fn.endswith(".safetensors"):
            sd.update(load_file(os.path.join(path, fn)))
    sd = {k: v.float() for k, v in sd.items() if k.startswith("model.")}
    missing = set(weight_shapes(dims)) - set(sd)
    if missing:
        raise ValueError(f"{path}: missing weights {sorted(missing)[:5]} ...")
    return dims, sd


def load_model_dir(path: str) -> Tuple[ModelDims, Dict[str, torch.Tensor]]:
    """A local model directory: CTranslate2 (model.bin) or HF (config.json + *.safetensors)."""
    if os.path.isfile(os.path.join(path, "model.bin")):
        from .ct2 import load_ct2_dir
        dims, sd, _ = load_ct2_dir(path)
        return dims, sd
    return load_hf_dir(path)


def resolve_model(model_size_or_path: str, seed: int = 0, eot_after: Optional[int] = None
                  ) -> Tuple[ModelDims, Dict[str, torch.Tensor], Optional[str]]:
    """-> (dims, float32 CPU state dict, model directory or None)."""
    spec = model_size_or_path
    if spec.startswith("synthetic:"):
        # synthetic:<name>[:<seed>][:margin]  ("margin": the decisive planted program, plant_margin)
        parts = spec.split(":")
        name = parts[1]
        plant = None
        if parts[-1] in ("margin", "margin_var"):
            plant = parts[-1]
            parts = parts[:-1]
        if len(parts) > 2:
            seed = int(parts[2])
        dims = model_dims(name)
        return dims, synthetic_state_dict(dims, seed, eot_after, plant=plant), None
    if os.path.isdir(spec):
        dims, sd = load_model_dir(spec)
        return dims, sd, spec
    env = os.environ.get("VLOG_AMD_MODEL_DIR_" + spec.replace("-", "_").replace(".", "_"))
    root = os.environ.get("VLOG_AMD_MODEL_ROOT")
    for cand in [env, os.path.join(root, spec) if root else None]:
        if cand and os.path.isdir(cand):
            dims, sd = load_model_dir(cand)
            return dims, sd, cand
    raise ValueError(
        f"model {spec!r}: no local weights (set VLOG_AMD_MODEL_DIR_<name> or VLOG_AMD_MODEL_ROOT, pass a "
        f"directory, or use 'synthetic:<name>'); downloading is not supported")
