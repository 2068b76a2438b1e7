"""sample_from_logits with the reference's signature (zonos/sampling.py:117-182) on the HIP sampler
kernel (zmi_sample_logits, the same code as the decode step's sampler).

Greedy decoding (temperature 0) is exact: repetition penalty, then argmax with first-index ties.
Stochastic sampling draws the exponential race's noise q from a counter-based hash seeded from
torch's global RNG, so torch.manual_seed() controls it as it controls the reference; pass `noise`
(the reference's q, sampling.py:20) to reproduce a reference draw exactly.
"""
from __future__ import annotations


import torch

from . import _lib


def sample_from_logits(logits: torch.Tensor, temperature: float = 1.0, top_p: float = 0.0, top_k: int = 0,
                       min_p: float = 0.0, linear: float = 0.0, conf: float = 0.0, quad: float = 0.0,
                       generated_tokens: torch.Tensor | None = None, repetition_penalty: float = 3.0,
                       repetition_penalty_window: int = 2, noise: torch.Tensor | None = None) -> torch.Tensor:
    """logits [B, 9, V] -> tokens [B, 9, 1] int64 (device tensors). V = 1025 (unpadded heads), 1026 (the
    reference's padded heads) or wider (pad_vocab_to_multiple_of, model.py:37,46-51) with every column past
    1025 at -inf, as _compute_logits leaves them (model.py:115): those never win, so they are dropped."""
    if logits.dim() != 3 or logits.shape[1] != 9 or logits.shape[2] < 1025:
        raise ValueError("logits must be [B, 9, V] with V >= 1025")
    dev = logits.device
    if dev.type != "cuda":
        raise ValueError("the HIP sampler takes device tensors")
    b, v = logits.shape[0], logits.shape[2]
    if v == 1025:  # the kernel's row is 1026 wide: the missing column can never be drawn
        logits = torch.cat([logits.float(), torch.full((b, 9, 1), float("-inf"), device=dev)], dim=-1)
    elif v > 1026:
        if not bool(torch.isneginf(logits[..., 1026:]).all()):
            raise ValueError("logits past column 1025 must be -inf (the HIP sampler draws from 1026 columns)")
        logits = logits[..., :1026]
    if noise is not None and noise.shape[-1] != 1026:
        noise = noise[..., :1026] if noise.shape[-1] > 1026 else torch.cat(
            [noise.float(), torch.ones(b, 9, 1026 - noise.shape[-1], device=noise.device)], dim=-1)
    # the reference draws its noise only when sampling (sampling.py:20-21); greedy leaves torch's RNG alone
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if temperature > 0 else 0
    prm = _lib.Sampling(float(temperature), float(top_p), float(min_p), float(linear), float(conf), float(quad),
                        float(repetition_penalty), 1.0, int(top_k), int(repetition_penalty_window), seed)
    p_dev = torch.tensor(bytearray(prm), dtype=torch.uint8).to(dev)
    lg = logits.to(torch.float32).contiguous()
    gen, gl = None, 0
    if generated_tokens is not None and generated_tokens.shape[-1] > 0:
        gen = generated_tokens.to(dev, torch.int32)
        if v == 1025:  # the reference clamps to logits.shape[-1] - 1 (sampling.py:111): the mask token 1025
            gen = gen.clamp_max(1024)  # penalises EOS (1024), not the padding column this wrapper adds
        gen = gen.contiguous()
        gl = gen.shape[-1]
    nz = None if noise is None else noise.to(dev, torch.float32).contiguous()
    out = torch.empty(b, 9, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().zmi_sample_logits(lg.data_ptr(), _lib.ptr(gen), gl, b, p_dev.data_ptr(), _lib.ptr(nz),
                                            out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream),
               "sample_logits")
    return out.to(torch.int64).unsqueeze(-1)


__all__ = ["sample_from_logits"]
