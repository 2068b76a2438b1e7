"""Repetition-penalty windows beyond the default 2 (sampling.py:99-114, 117-182), by the REFERENCE.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_penalty.py

Writes tests/golden/penalty_windows.safetensors: bf16-valued logits with ties, a 40-frame
history with repeated tokens, and the reference's penalised logits and greedy choice for the
windows 1, 2, 8, 16, 40 (whole history), 0 (the slice [..., -0:], also the whole history) and
-3 (the slice [..., 3:]).
"""
from __future__ import annotations

import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference, save  # noqa: E402

WINDOWS = [1, 2, 8, 16, 40, 0, -3]


def main():
    _, zs, _, _, _ = import_reference()
    g = torch.Generator().manual_seed(7)
    lg = (torch.randn(2, 9, 1026, generator=g) * 2).to(torch.bfloat16).float()
    lg[..., 1025] = -torch.inf
    lg[:, 1:, 1024] = -torch.inf
    gen = torch.randint(0, 40, (2, 9, 40), generator=g)  # small alphabet: many repeats
    gen[:, :, 5:9] = 1025                                 # mask tokens clamp to the last column
    tens = {"logits": lg, "generated": gen}
    for w in WINDOWS:
        tens[f"pen{w}"] = zs.modify_logit_for_repetition_penalty(lg.clone(), gen, 3.0, w)
        tens[f"greedy{w}"] = zs.sample_from_logits(lg.clone(), temperature=0.0, generated_tokens=gen,
                                                   repetition_penalty=3.0, repetition_penalty_window=w)
    save("penalty_windows", tens, {"windows": WINDOWS, "penalty": 3.0})


if __name__ == "__main__":
    main()
