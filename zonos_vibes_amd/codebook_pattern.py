"""apply_delay_pattern / revert_delay_pattern with the reference's signatures
(zonos/codebook_pattern.py:5-12), on the HIP kernels (zmi_apply_delay_pattern / zmi_revert_delay_pattern).

generate() keeps its delayed codes on the device in the engine's slot state (zmi_delay_init /
zmi_delay_revert); these are the standalone forms for callers of the reference's module.
"""
from __future__ import annotations

import torch

from . import _lib


def _run(fn, codes: torch.Tensor, t_out: int, *extra) -> torch.Tensor:
    if codes.device.type != "cuda":
        raise ValueError("the HIP delay-pattern kernels take device tensors")
    c = codes.to(torch.int64).contiguous()
    out = torch.empty(c.shape[0], c.shape[1], t_out, dtype=torch.int64, device=c.device)
    if out.numel():
        _lib.check(fn(c.data_ptr(), out.data_ptr(), c.shape[0], c.shape[2], *extra,
                      torch.cuda.current_stream(c.device).cuda_stream), "delay pattern")
    return out


def apply_delay_pattern(codes: torch.Tensor, mask_token: int) -> torch.Tensor:
    """[B, 9, T] -> [B, 9, T + 9]: codebook k shifted right by k + 1, padded with mask_token."""
    if codes.shape[1] != 9:
        raise ValueError("9 codebooks expected")
    return _run(_lib.lib().zmi_apply_delay_pattern, codes, codes.shape[2] + 9, int(mask_token))


def revert_delay_pattern(codes: torch.Tensor) -> torch.Tensor:
    """[B, 9, T] -> [B, 9, T - 9]: codebook k keeps positions k + 1 .. T - 9 + k."""
    if codes.shape[1] != 9 or codes.shape[2] < 9:
        raise ValueError("[B, 9, T >= 9] expected")
    return _run(_lib.lib().zmi_revert_delay_pattern, codes, codes.shape[2] - 9)
