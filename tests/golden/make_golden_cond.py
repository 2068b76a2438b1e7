"""Golden fixture for the prefix conditioner, produced by the REFERENCE (in this container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_cond.py

Imports the reference through make_golden.import_reference() (stubbed text/audio front-end), builds
its `PrefixConditioner` (zonos/conditioning.py:284-310) in bf16 at d = 256 with the
Zonos-v0.1-transformer conditioner list plus the hybrid-only ones, fills every parameter from a
seeded generator, and records `torch.cat([pc(cond), pc(uncond)])` (zonos/model.py:204-212) for a few
cond dicts built by the reference's own `make_cond_dict` (:326-395). `phonemize` (the eSpeak
front-end, out of scope) is replaced by the identity, so the "text" IS the phoneme string and the
reference's own `tokenize_phonemes` runs. Weights, inputs and outputs go into
tests/golden/prefix_cond.safetensors (data only).
"""
from __future__ import annotations

import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from make_golden import import_reference, save  # noqa: E402

D = 256
CONDITIONERS = [
    {"type": "EspeakPhonemeConditioner", "name": "espeak"},
    {"type": "PassthroughConditioner", "name": "speaker", "cond_dim": 128, "uncond_type": "learned",
     "projection": "linear"},
    {"type": "FourierConditioner", "name": "emotion", "input_dim": 8, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "fmax", "min_val": 0, "max_val": 24000, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "pitch_std", "min_val": 0, "max_val": 400, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "speaking_rate", "min_val": 0, "max_val": 40, "uncond_type": "learned"},
    {"type": "IntegerConditioner", "name": "language_id", "min_val": -1, "max_val": 126, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "vqscore_8", "input_dim": 8, "min_val": 0.5, "max_val": 0.8,
     "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "ctc_loss", "min_val": -1.0, "max_val": 1000, "uncond_type": "learned"},
    {"type": "FourierConditioner", "name": "dnsmos_ovrl", "min_val": 1, "max_val": 5, "uncond_type": "learned"},
    {"type": "IntegerConditioner", "name": "speaker_noised", "min_val": 0, "max_val": 1, "uncond_type": "learned"},
]

CASES = [
    dict(tag="default", text="həloʊ, wɜːld!", language="en-us", kw={}),
    dict(tag="unknown_symbols", text="ˈʃeː 7 ŋ'xyz★", language="de",
         kw=dict(fmax=24000.0, pitch_std=120.0, speaking_rate=28.0, emotion=[1, 0, 0, 0, 0, 0, 0.5, 0.2],
                 unconditional_keys=set())),
    dict(tag="uncond_speaker", text="a", language="ja", kw=dict(unconditional_keys={"speaker", "emotion"},
                                                               speaker_noised=True)),
]


def main():
    zm, zs, zc, ZonosConfig, BACKBONES = import_reference()
    cond_mod = sys.modules["zonos.conditioning"]
    from zonos.config import PrefixConditionerConfig
    cond_mod.phonemize = lambda texts, languages: list(texts)
    torch.set_num_threads(8)

    pc = cond_mod.PrefixConditioner(PrefixConditionerConfig(conditioners=CONDITIONERS, projection="none"), D)
    pc = pc.to(torch.bfloat16)
    g = torch.Generator().manual_seed(3)
    tensors = {}
    with torch.no_grad():
        for name, t in list(pc.state_dict().items()):
            if name.startswith("norm.weight"):
                v = 1.0 + 0.1 * torch.randn(t.shape, generator=g)
            elif name.startswith("norm.bias"):
                v = 0.1 * torch.randn(t.shape, generator=g)
            else:
                v = torch.randn(t.shape, generator=g)
            t.copy_(v.to(t.dtype))
            tensors["w/" + name] = t.clone()
    speaker = (0.5 * torch.randn(1, 128, generator=g)).to(torch.bfloat16)
    tensors["speaker"] = speaker
    meta = {"d": D, "conditioners": CONDITIONERS, "cases": []}
    for c in CASES:
        kw = dict(c["kw"])
        kw.setdefault("speaker", speaker)
        cd = cond_mod.make_cond_dict(text=c["text"], language=c["language"], device="cpu", **kw)
        uncond = {k: cd[k] for k in pc.required_keys}
        with torch.inference_mode():
            out = torch.cat([pc(cd), pc(uncond)])
        ids, lengths = cond_mod.tokenize_phonemes([c["text"]])
        tensors[c["tag"] + "/out"] = out
        tensors[c["tag"] + "/ids"] = ids
        mkw = {k: (sorted(v) if isinstance(v, set) else v) for k, v in kw.items() if k != "speaker"}
        meta["cases"].append(dict(tag=c["tag"], text=c["text"], language=c["language"], kw=mkw,
                                  keys=sorted(cd.keys())))
    save("prefix_cond", tensors, json.loads(json.dumps(meta)))


if __name__ == "__main__":
    main()
