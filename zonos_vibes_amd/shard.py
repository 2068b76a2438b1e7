"""Utterance sharding across GPUs of one node.

Utterances are independent (own KV rows, own EOS state machine, own sampler seed), so a batch is
partitioned over ranks with no data-path collective: one process per GPU, each holding a full weight
replica, each running its shard through `Zonos.generate_batch` (continuous batching over engine
slots). The only collective is the optional end-of-batch gather of the codes to one rank, as int16
([9, T] per utterance, values in [0, 1025]) over RCCL/xGMI on the GPU box (int32 on gloo, which has
no int16 collectives, in the CPU tests).

Assignment is longest-processing-time first by estimated frames (the reference runs one utterance
per call, `model.py:218-231`; its callers loop over utterances, `sample.py:18-20`,
`server.py:124-134`), deterministic in the inputs only, so every rank computes the same plan
without communicating. Result i equals `generate()` on utterance i whatever the rank count
(tests/test_shard.py checks this bit-exactly against the single-process run).
"""
from __future__ import annotations

from typing import Protocol, Sequence

import torch

N_CODEBOOKS = 9


class BatchGenerator(Protocol):
    def generate_batch(self, conds, prefixes=None, max_new_tokens=..., cfg_scale=2.0, sampling_params=...,
                       seeds=None, **kw) -> list[torch.Tensor]: ...


def estimated_frames(conds: Sequence[torch.Tensor], prefixes: Sequence[torch.Tensor | None],
                     max_new_tokens: Sequence[int]) -> list[int]:
    """Decode cost proxy per utterance: steps (N + 8) plus the prefill rows it re-reads (Lc + P + 1)."""
    out = []
    for c, p, n in zip(conds, prefixes, max_new_tokens):
        plen = 0 if p is None else p.shape[-1]
        out.append(int(n) + 8 + c.shape[1] + plen + 1)
    return out


def lpt_assign(costs: Sequence[int], world: int) -> list[list[int]]:
    """Greedy LPT: utterances by decreasing cost (ties: lower index first) onto the least-loaded rank
    (ties: lower rank). Each rank's list is returned in ascending utterance order."""
    if world < 1:
        raise ValueError("world must be >= 1")
    loads = [0] * world
    parts: list[list[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda r: (loads[r], r))
        parts[r].append(i)
        loads[r] += costs[i]
    return [sorted(p) for p in parts]


def _rank_world(group=None) -> tuple[int, int]:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def gather_codes(local: Sequence[torch.Tensor], local_idx: Sequence[int], n_total: int, dst: int = 0,
                 group=None, device: torch.device | str = "cpu") -> list[torch.Tensor] | None:
    """End-of-batch gather: every rank's [1, 9, T_i] codes to rank `dst`, in global utterance order.

    Two all_gathers of fixed-shape tensors (int64 sizes, then the padded 2-byte code payload), so it runs
    unchanged on RCCL (device tensors) and gloo (CPU tensors). Returns the full list on `dst`, None
    elsewhere."""
    rank, world = _rank_world(group)
    if world == 1:
        out: list[torch.Tensor | None] = [None] * n_total
        for i, c in zip(local_idx, local):
            out[i] = c
        return out  # type: ignore[return-value]
    return _gather_collective(local, local_idx, n_total, dst, group, device, rank, world)


def _gather_collective(local, local_idx, n_total, dst, group, device, rank, world):
    """gather_codes' collective path (any world size, including 1 in tests: the RCCL int16 hand-off on one GPU)."""
    import torch.distributed as dist
    lens = [int(c.shape[-1]) for c in local]
    meta = torch.tensor([len(local), sum(lens)] + [v for i, t in zip(local_idx, lens) for v in (i, t)],
                        dtype=torch.int64)
    hdr = torch.tensor([meta.numel()], dtype=torch.int64, device=device)
    hdrs = [torch.zeros_like(hdr) for _ in range(world)]
    dist.all_gather(hdrs, hdr, group=group)
    mmax = max(int(h.item()) for h in hdrs)
    meta_p = torch.zeros(mmax, dtype=torch.int64, device=device)
    meta_p[:meta.numel()] = meta.to(device)
    metas = [torch.zeros_like(meta_p) for _ in range(world)]
    dist.all_gather(metas, meta_p, group=group)
    tmax = max(int(m[1].item()) for m in metas)
    # 2-byte payload on RCCL: the codes as int16 bit patterns, gathered as a bfloat16 view (RCCL / NCCL have no int16
    # type; all_gather copies bytes, so any 2-byte type carries them exactly); gloo carries int32
    nccl = dist.get_backend(group) == "nccl"
    wire = torch.int16 if nccl else torch.int32
    flat = torch.zeros(N_CODEBOOKS, max(tmax, 1), dtype=wire, device=device)
    if local:
        cat = torch.cat([c.reshape(N_CODEBOOKS, -1) for c in local], dim=1)
        if cat.min() < 0 or cat.max() > 1025:
            raise ValueError("codes out of the int16 hand-off range [0, 1025]")
        flat[:, :cat.shape[1]] = cat.to(device=device, dtype=wire)
    flats = [torch.zeros_like(flat) for _ in range(world)]
    if nccl:
        dist.all_gather([f.view(torch.bfloat16) for f in flats], flat.view(torch.bfloat16), group=group)
    else:
        dist.all_gather(flats, flat, group=group)
    if rank != dst:
        return None
    out = [None] * n_total
    for m, f in zip(metas, flats):
        m = m.cpu().tolist()
        col = 0
        for j in range(m[0]):
            i, t = m[2 + 2 * j], m[3 + 2 * j]
            out[i] = f[:, col:col + t].to(torch.int64).unsqueeze(0)
            col += t
    missing = [i for i, c in enumerate(out) if c is None]
    if missing:
        raise RuntimeError(f"gather_codes: utterances {missing} were produced by no rank")
    return out  # type: ignore[return-value]


def generate_sharded(model: BatchGenerator, conds: Sequence[torch.Tensor],
                     prefixes: Sequence[torch.Tensor | None] | None = None,
                     max_new_tokens: Sequence[int] | int = 86 * 30, cfg_scale: float = 2.0,
                     sampling_params: dict = dict(min_p=0.1), seeds: Sequence[int] | None = None,
                     gather: bool = True, dst: int = 0, group=None, gather_device: torch.device | str = "cpu",
                     **kw) -> tuple[list[int], list[torch.Tensor], list[torch.Tensor] | None]:
    """Run this rank's LPT shard of the batch; optionally gather all codes on `dst`.

    `seeds` must be given for stochastic sampling when world > 1 (every rank must agree on utterance
    i's seed; a rank-local draw would not). Returns (my utterance indices, my codes, gathered codes on
    `dst` or None)."""
    rank, world = _rank_world(group)
    n = len(conds)
    prefixes = list(prefixes) if prefixes is not None else [None] * n
    mnt = [max_new_tokens] * n if isinstance(max_new_tokens, int) else list(max_new_tokens)
    if seeds is None:
        if world > 1 and float(dict(sampling_params).get("temperature", 1.0)) > 0:
            raise ValueError("generate_sharded: pass explicit per-utterance seeds for stochastic sampling")
        seeds = list(range(n))
    mine = lpt_assign(estimated_frames(conds, prefixes, mnt), world)[rank]
    local: list[torch.Tensor] = []
    if mine:
        local = model.generate_batch([conds[i] for i in mine], [prefixes[i] for i in mine],
                                     max_new_tokens=[mnt[i] for i in mine], cfg_scale=cfg_scale,
                                     sampling_params=sampling_params, seeds=[seeds[i] for i in mine], **kw)
    gathered = gather_codes(local, mine, n, dst, group, gather_device) if gather else None
    return mine, local, gathered


__all__ = ["estimated_frames", "lpt_assign", "gather_codes", "generate_sharded"]
