"""The reference's backbone plugin seam (zonos/backbone/__init__.py:1-12; the contract of
TorchZonosBackbone, zonos/backbone/_torch.py:52-80) on the HIP kernels: BACKBONES["hip"].

    bb = BACKBONES["hip"](config.backbone)              # BackboneConfig
    bb.load_state_dict(sd)                              # TorchZonosBackbone names: layers.{i}..., norm_f.*
    cache = bb.allocate_inference_cache(B, max_seqlen)  # {layer: (K, V^T)}
    params = InferenceParams(max_seqlen, B, key_value_memory_dict=cache,
                             lengths_per_sample=torch.zeros(B, dtype=torch.int32, device="cuda"))
    y = bb.forward(hidden_states, params)               # [B, S, d] -> [B, S, d], norm_f applied

forward runs every layer on the same kernels as generate()'s prefill (LayerNorm-prologue GEMVs,
RoPE + KV-write epilogue, blocked attention, SwiGLU, residual epilogues), then norm_f. Positions
are lengths_per_sample + arange(S) (_torch.py:74-77), and each row's K/V are written at those
positions (the reference writes its cache at seqlen_offset, equal to them in every caller).
generate() does not go through this seam: it fuses across it (heads, sampler, frame state), so
this class is the drop-in for callers that use the backbone alone.
"""
from __future__ import annotations

import torch

from . import _lib
from .config import BackboneConfig, InferenceParams, PrefixConditionerConfig, ZonosConfig
from .engine import HipEngine, make_engine


class HipZonosBackbone:
    supported_architectures = ["transformer", "hybrid"]

    def __init__(self, config: BackboneConfig, device="cuda"):
        self.config = config
        self.device = torch.device(device)
        self._cfg = ZonosConfig(config, PrefixConditionerConfig([], "none"))
        self._sd = None
        self.engine: HipEngine | None = None

    def load_state_dict(self, sd: dict):
        """TorchZonosBackbone parameter names (layers.{i}.norm/mixer/norm2/mlp..., norm_f.*)."""
        self._sd = {"backbone." + k: v for k, v in sd.items()}
        if self.engine is not None:
            self.engine.load_state_dict(self._sd)

    def allocate_inference_cache(self, batch_size: int, max_seqlen: int, dtype=torch.bfloat16) -> dict:
        """{layer: (K [B][Hkv][Smax][hd], V^T [B][Hkv][hd][Smax])} bf16 (_torch.py:64-71); for the hybrid
        (_mamba_ssm.py:38-42) Mamba2 layers hold (conv ring, SSM state) instead."""
        if dtype != torch.bfloat16:
            raise ValueError("the HIP backbone keeps its KV cache in bf16 (as the reference's generate does)")
        slots = (batch_size + 1) // 2
        self.engine = make_engine(self._cfg, self.device, max_slots=slots, max_seqlen=max_seqlen,
                                  max_prefill=slots * max_seqlen)
        if self._sd is not None:
            self.engine.load_state_dict(self._sd)
        e = self.engine
        if e.hybrid:
            return e.inference_cache()
        return {i: (e.kc[i], e.vc[i]) for i in range(e.L)}

    def forward(self, hidden_states: torch.Tensor, inference_params: InferenceParams) -> torch.Tensor:
        e = self.engine
        if e is None or e.w is None:
            raise RuntimeError("allocate_inference_cache() and load_state_dict() first")
        b, s, d = hidden_states.shape
        m = b * s
        if m > 2 * e.max_prefill or b > e.R:
            raise ValueError("batch x length exceeds the allocated inference cache")
        lengths = inference_params.lengths_per_sample
        if lengths is None:
            lengths = torch.full((b,), inference_params.seqlen_offset, dtype=torch.int32, device=self.device)
        # K / V are written (and RoPE'd) at lengths_per_sample + arange(S) (_torch.py:74-77): bound those
        l_max, l_min = (int(v) for v in torch.stack([lengths.max(), lengths.min()]).tolist())
        max_pos = max(l_max, inference_params.seqlen_offset) + s - 1
        if l_min < 0:
            raise ValueError("negative lengths_per_sample")
        if max_pos >= e.smax:
            raise ValueError("positions beyond the allocated max_seqlen")
        if e.hybrid and (inference_params.seqlen_offset or l_max):
            raise NotImplementedError("hybrid backbone plugin: prefill from position 0 only (decode runs inside "
                                      "generate(), whose step fuses the heads and sampler)")
        e.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(e.stream):
            e.x_pre[:m] = hidden_states.reshape(m, d).to(torch.bfloat16)
            pos = lengths.to(self.device, torch.int32).view(b, 1) + torch.arange(s, dtype=torch.int32,
                                                                                device=self.device).view(1, s)
            e.row_pos_pre[:m] = pos.reshape(m)
            e.row_kv_pre[:m] = torch.arange(b, dtype=torch.int32, device=self.device).repeat_interleave(s)
            e._prefill_layers(m, max_pos)
            out = torch.empty(m, d, dtype=torch.bfloat16, device=self.device)
            e.final_norm_pre(m, out)
        torch.cuda.current_stream(self.device).wait_stream(e.stream)
        e.check_errors()
        return out.view(b, s, d)

    __call__ = forward


BACKBONES = {"hip": HipZonosBackbone}

__all__ = ["BACKBONES", "HipZonosBackbone", "InferenceParams"]
