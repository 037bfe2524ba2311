import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from oracle import transcribe as otr, mel as omel
from oracle.model import OracleWhisper
from vlog_amd.audio import speech_like
from vlog_amd.transcribe import WhisperModel
from vlog_amd.tokenizer import Tokenizer
from vlog_amd.weights import round_bf16, synthetic_state_dict
model = WhisperModel("synthetic:tiny:3", device="cuda", eot_after=60)
x = np.concatenate([speech_like(30.0, 300), speech_like(25.0, 301), speech_like(14.0, 302)])
x = (np.clip(np.round(x * 32768), -32768, 32767).astype(np.int16).astype(np.float32) / 32768)
segs, info = model.transcribe(x, language=None, beam_size=5)
for s in segs:
    print("GPU", s.seek, round(s.start, 2), round(s.end, 2), s.temperature, round(s.avg_logprob, 3), round(s.no_speech_prob, 4), len(s.tokens), s.tokens[:6], s.text[:40])
orc = OracleWhisper(round_bf16(synthetic_state_dict(model.dims, seed=3, eot_after=60)), model.dims, np.float32)
feats = model.engine.features(torch.from_numpy(x)).cpu().numpy()
def enc(win):
    return model.engine.encode(torch.from_numpy(np.ascontiguousarray(win)).cuda(), [0], [3000]).float().cpu().numpy()
ref, lang = otr.transcribe(orc, lambda l: Tokenizer(model.dims, language=l), x, beam_size=5, encoder=enc, features=feats)
for s in ref:
    print("ORC", round(s["start"], 2), round(s["end"], 2), s["temperature"], round(s["avg_logprob"], 3), round(s["no_speech_prob"], 4), len(s["tokens"]), s["tokens"][:6], s["text"][:40])
print(info.language, lang)
