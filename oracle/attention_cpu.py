"""ORACLE — the reference's decode / prefill attention arithmetic, restated. TEST INFRASTRUCTURE ONLY.

The reference calls F.scaled_dot_product_attention(q, k, v, is_causal=s > 1, enable_gqa=True) on
bf16 CPU tensors (zonos/backbone/_torch.py:136). ATen runs that on its CPU flash-attention kernel,
whose numerics (block size and rounding points) are:

    s_k = fp32(q . K_k) * scale                       (scores GEMM in fp32, then the scale)
    per 512-key block j:  M_j = max(M_{j-1}, max_{k in j} s_k)
                          e_k = exp(s_k - M_j);  P_k = bf16(e_k)
                          l   = sum_{k in j} e_k + exp(M_{j-1} - M_j) * l
                          acc = acc * exp(M_{j-1} - M_j) + sum_{k in j} P_k V_k     (fp32)
    out = bf16(acc * (1 / l))

This module restates that per query (dot products in float64 and then rounded to fp32, so the
only remaining difference to any fp32 implementation is the accumulation order). It is pinned
against torch's own CPU SDPA in tests/test_oracle_golden.py (block 512 with bf16 P reproduces it
far better than an fp32-P or an unblocked softmax), and is the reference the HIP attention kernel
(zonos_vibes_amd/csrc/zmi_attn.hip) is compared with in tests/test_gpu_kernels.py.
"""
from __future__ import annotations

import math

import torch

BLOCK = 512


def attend_row(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, block: int = BLOCK,
               round_p: bool = True) -> torch.Tensor:
    """q [hd], k/v [n, hd] (bf16) -> [hd] bf16: one query head over n keys."""
    scale = torch.tensor(1.0 / math.sqrt(q.shape[0]), dtype=torch.float32)
    s_all = (k.double() @ q.double()).float() * scale
    m = torch.tensor(-math.inf)
    l = torch.tensor(0.0)
    acc = torch.zeros(q.shape[0])
    for n0 in range(0, k.shape[0], block):
        s = s_all[n0:n0 + block]
        mn = torch.maximum(m, s.max())
        e = torch.exp(s - mn)
        et = torch.exp(m - mn)
        l = e.double().sum().float() + et * l
        p = e.to(torch.bfloat16).double() if round_p else e.double()
        acc = acc * et + (p @ v[n0:n0 + block].double()).float()
        m = mn
    return (acc * (torch.tensor(1.0) / l)).to(torch.bfloat16)


def attend(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, pos: int, **kw) -> torch.Tensor:
    """GQA for one query at position `pos`: q [hq, hd], k/v [hkv, >pos, hd] -> [hq, hd] bf16."""
    hq, hkv = q.shape[0], k.shape[0]
    g = hq // hkv
    return torch.stack([attend_row(q[h], k[h // g, : pos + 1], v[h // g, : pos + 1], **kw) for h in range(hq)])
