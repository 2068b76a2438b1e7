"""Model configuration mirror of the reference's `zonos/config.py`.

Same dataclass names and field meanings as the reference so that a `config.json`
written for `Zonos.from_local` (reference `zonos/model.py:65-88`) loads unchanged:

* `InferenceParams`         -> reference `zonos/config.py:8-25`
* `BackboneConfig`          -> reference `zonos/config.py:28-39`
* `PrefixConditionerConfig` -> reference `zonos/config.py:42-45`
* `ZonosConfig.from_dict`   -> reference `zonos/config.py:48-62`

Only the fields the hot path reads are interpreted; the prefix conditioner's list is read by
`zonos_vibes_amd.conditioning.PrefixConditioner`.
"""
from __future__ import annotations

from dataclasses import dataclass, field, asdict
from typing import Any

# Token constants of the 44.1 kHz DAC codebooks (reference `zonos/config.py:50-52`).
N_CODEBOOKS = 9
CODEBOOK_SIZE = 1024
EOS_TOKEN = 1024
MASK_TOKEN = 1025
EMB_VOCAB = 1026          # nn.Embedding(1026, d)   reference model.py:36
HEAD_VOCAB = 1025         # nn.Linear(d, 1025)      reference model.py:37
HEAD_VOCAB_PADDED = 1026  # pad_weight_ adds 1025 % 8 = 1 zero row (utils.py:12-27)
DAC_HOP = 512
DAC_SAMPLE_RATE = 44100
ROPE_TABLE_LEN = 16384    # precompute_freqs_cis(16384, hd)  reference _torch.py:67


@dataclass
class InferenceParams:
    """Decode state handed to a backbone's forward (reference zonos/config.py:8-25)."""
    max_seqlen: int
    max_batch_size: int
    seqlen_offset: int = 0
    batch_size_offset: int = 0
    key_value_memory_dict: dict = field(default_factory=dict)
    lengths_per_sample: Any = None

    def reset(self, max_seqlen: int, max_batch_size: int):
        self.max_seqlen = max_seqlen
        self.max_batch_size = max_batch_size
        self.seqlen_offset = 0
        if self.lengths_per_sample is not None:
            self.lengths_per_sample.zero_()


@dataclass
class BackboneConfig:
    d_model: int = 1024
    d_intermediate: int = 0
    attn_mlp_d_intermediate: int = 0
    n_layer: int = 16
    ssm_cfg: dict = field(default_factory=dict)
    attn_layer_idx: list = field(default_factory=list)
    attn_cfg: dict = field(default_factory=dict)
    rms_norm: bool = False
    residual_in_fp32: bool = False
    norm_epsilon: float = 1e-5

    @property
    def num_heads(self) -> int:
        return int(self.attn_cfg["num_heads"])

    @property
    def num_heads_kv(self) -> int:
        return int(self.attn_cfg["num_heads_kv"])

    @property
    def head_dim(self) -> int:
        return self.d_model // self.num_heads

    @property
    def is_hybrid(self) -> bool:
        return bool(self.ssm_cfg)

    def mamba2_dims(self) -> dict:
        """Mamba2 mixer geometry from ssm_cfg with mamba-ssm 2.2.4's Mamba2 defaults (d_state 128,
        d_conv 4, expand 2, headdim 64, ngroups 1): d_ssm = expand d_model, nheads = d_ssm / headdim,
        in_proj width 2 d_ssm + 2 ngroups d_state + nheads (mamba_ssm/modules/mamba2.py)."""
        c = dict(self.ssm_cfg)
        if c.get("layer", "Mamba1") != "Mamba2":
            raise NotImplementedError("only Mamba2 mixers are built (Zonos-v0.1-hybrid uses ssm_cfg layer=Mamba2)")
        d_ssm = int(c.get("d_ssm") or c.get("expand", 2) * self.d_model)
        hd = int(c.get("headdim", 64))
        out = dict(d_ssm=d_ssm, headdim=hd, nheads=d_ssm // hd, d_state=int(c.get("d_state", 128)),
                   d_conv=int(c.get("d_conv", 4)), ngroups=int(c.get("ngroups", 1)),
                   rmsnorm=bool(c.get("rmsnorm", True)), norm_before_gate=bool(c.get("norm_before_gate", False)),
                   D_has_hdim=bool(c.get("D_has_hdim", False)))
        out["conv_dim"] = d_ssm + 2 * out["ngroups"] * out["d_state"]
        out["d_in_proj"] = 2 * d_ssm + 2 * out["ngroups"] * out["d_state"] + out["nheads"]
        return out


@dataclass
class PrefixConditionerConfig:
    conditioners: list = field(default_factory=list)
    projection: str = "none"


@dataclass
class ZonosConfig:
    backbone: BackboneConfig
    prefix_conditioner: PrefixConditionerConfig
    eos_token_id: int = EOS_TOKEN
    masked_token_id: int = MASK_TOKEN
    pad_vocab_to_multiple_of: int = 8

    @classmethod
    def from_dict(cls, d: dict) -> "ZonosConfig":
        d = dict(d)
        bb = BackboneConfig(**d.pop("backbone"))
        pc = PrefixConditionerConfig(**d.pop("prefix_conditioner", {"conditioners": [], "projection": "none"}))
        return cls(bb, pc, **d)

    def to_dict(self) -> dict[str, Any]:
        return asdict(self)


def transformer_config(d_model: int, n_layer: int, num_heads: int, num_heads_kv: int, d_ff: int,
                       eps: float = 1e-5) -> ZonosConfig:
    """A transformer-backbone `ZonosConfig` (the `torch` backbone, reference _torch.py:52-80)."""
    bb = BackboneConfig(
        d_model=d_model, d_intermediate=0, attn_mlp_d_intermediate=d_ff, n_layer=n_layer, ssm_cfg={},
        attn_layer_idx=[], attn_cfg={"causal": True, "num_heads": num_heads, "num_heads_kv": num_heads_kv,
                                     "rotary_emb_dim": d_model // num_heads},
        rms_norm=False, residual_in_fp32=False, norm_epsilon=eps)
    return ZonosConfig(bb, PrefixConditionerConfig([], "none"))


def zonos_v01_transformer() -> ZonosConfig:
    """Zonos-v0.1-transformer dims (d=2048, L=26, H=16/4, FFN=8192)."""
    return transformer_config(2048, 26, 16, 4, 8192)


def tiny_transformer(n_layer: int = 2) -> ZonosConfig:
    """Small config used by the parity fixtures (head_dim stays 128, GQA group 4)."""
    return transformer_config(512, n_layer, 4, 1, 1024)


def hybrid_config(d_model: int, n_layer: int, attn_layer_idx: list, num_heads: int, num_heads_kv: int,
                  d_intermediate: int = 0, attn_mlp_d_intermediate: int = 0, eps: float = 1e-5) -> ZonosConfig:
    """A hybrid-backbone `ZonosConfig` (reference MambaSSMZonosBackbone, _mamba_ssm.py:9-57): Mamba2 mixers,
    MHA mixers at attn_layer_idx (mamba_ssm MHA: non-interleaved rotary over the whole head)."""
    bb = BackboneConfig(
        d_model=d_model, d_intermediate=d_intermediate, attn_mlp_d_intermediate=attn_mlp_d_intermediate,
        n_layer=n_layer, ssm_cfg={"layer": "Mamba2"}, attn_layer_idx=list(attn_layer_idx),
        attn_cfg={"causal": True, "num_heads": num_heads, "num_heads_kv": num_heads_kv,
                  "rotary_emb_dim": d_model // num_heads, "qkv_proj_bias": False, "out_proj_bias": False},
        rms_norm=False, residual_in_fp32=False, norm_epsilon=eps)
    return ZonosConfig(bb, PrefixConditionerConfig([], "none"))


def zonos_v01_hybrid() -> ZonosConfig:
    """Zonos-v0.1-hybrid dims as published in its config.json (d 2048, 46 layers, Mamba2 mixers, MHA 16/4
    heads at layers 9/18/27/36/45, no MLPs). Not verifiable offline (no checkpoint or config in the
    reference tree): the kernels take the dims from whatever config.json is loaded."""
    return hybrid_config(2048, 46, [9, 18, 27, 36, 45], 16, 4)


def tiny_hybrid(n_layer: int = 4, attn_layer_idx=(2,), d_intermediate: int = 0,
                attn_mlp_d_intermediate: int = 0) -> ZonosConfig:
    """Small hybrid for parity tests: d 512 (d_ssm 1024, 16 Mamba2 heads), MHA 4/1 heads x 128."""
    return hybrid_config(512, n_layer, list(attn_layer_idx), 4, 1, d_intermediate, attn_mlp_d_intermediate)


PRESETS = {
    "zonos-v0.1-transformer": zonos_v01_transformer,
    "zonos-v0.1-hybrid": zonos_v01_hybrid,
    "tiny": tiny_transformer,
    "tiny-hybrid": tiny_hybrid,
}
