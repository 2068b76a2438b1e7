"""ORACLE — greedy-parity criterion shared by tests/ and __graft_entry__.smoke(). TEST INFRASTRUCTURE ONLY.

Exact equality of greedy codes with the reference is only defined where the reference's own
decision is numerically determined: the reference is not bit-reproducible against itself
(CPU thread counts and torch.compile change its trajectories), its logits are
bf16-quantised head outputs (exact ties occur), and no GPU reduction order can reproduce the
CPU GEMM's bf16 rounding bit for bit. The criterion:

    the HIP trajectory equals the reference trajectory until the first decision whose
    reference margin (top-1 minus top-2 score, after CFG / EOS bias / repetition penalty)
    is within `floor_ulps` bf16 ulps of the top score.

Decisions before that point must match exactly; a divergence at a determined decision fails.
"""
from __future__ import annotations

import math

import torch

from .zonos_cpu import OracleZonos


def bf16_ulp(x: float) -> float:
    return 2.0 ** (math.floor(math.log2(max(abs(x), 1e-30))) - 7)


def greedy_divergence(gpu_delayed: torch.Tensor, oracle: OracleZonos, cond, prefix, n: int,
                      floor_ulps: float = 8.0):
    """Returns None if the delayed-code arrays are identical, else a dict describing the first
    divergence; raises AssertionError if that divergence happens at a determined decision."""
    trace: list = []
    oracle.generate(cond, prefix, max_new_tokens=n, sampling_params=dict(temperature=0.0), trace=trace)
    ref = oracle.last_delayed[0]
    got = gpu_delayed[:, : ref.shape[-1]].cpu().long()
    diff = got != ref
    if not diff.any():
        return None
    o = int(diff.any(dim=0).nonzero()[0])
    k = int(diff[:, o].nonzero()[0])
    p = 0 if prefix is None else prefix.shape[-1]
    step = o - (p + 1)
    fin = trace[step][0, k]
    top2 = fin.topk(2).values
    info = dict(position=o, codebook=k, step=step, margin=float(top2[0] - top2[1]), ulp=bf16_ulp(float(top2[0])))
    assert info["margin"] <= floor_ulps * info["ulp"], f"divergence at a numerically determined decision: {info}"
    return info
