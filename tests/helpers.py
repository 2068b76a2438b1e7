"""Shared test helpers: golden fixture loading and synthetic model construction."""
import json
import math
import os

import torch
from safetensors import safe_open

from zonos_vibes_amd import synthetic as syn
from zonos_vibes_amd.config import ZonosConfig

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    path = os.path.join(GOLDEN, name + ".safetensors")
    with safe_open(path, framework="pt") as f:
        meta = json.loads(f.metadata()["json"])
        tens = {k: f.get_tensor(k) for k in f.keys()}
    return tens, meta


def synthetic_weights(cfg: ZonosConfig, seed=0, zero_eos=False, eos_row_scale=None):
    w = dict(syn.iter_torch_cpu(syn.zonos_specs(cfg), seed))
    h0 = w["heads.0.weight"].clone()
    if zero_eos:
        h0[1024] = 0
    if eos_row_scale is not None:
        h0[1024] = (h0[1024].float() * eos_row_scale).to(torch.bfloat16)
    w["heads.0.weight"] = h0
    return w


def dac_weights(seed=0):
    return dict(syn.iter_torch_cpu(syn.dac_specs(), seed))


def synthetic_wav(b: int, n: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(n, dtype=torch.float64) / 44100.0
    out = []
    for _ in range(b):
        f = 80 + 900 * torch.rand(4, generator=g, dtype=torch.float64)
        a = 0.2 * torch.rand(4, generator=g, dtype=torch.float64)
        x = sum(a[i] * torch.sin(2 * math.pi * f[i] * t) for i in range(4))
        x = x + 0.02 * torch.randn(n, generator=g, dtype=torch.float64)
        out.append(x.clamp(-0.9, 0.9))
    return torch.stack(out).unsqueeze(1).float()
