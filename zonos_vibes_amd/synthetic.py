"""Counter-based synthetic weights and inputs (no checkpoints exist offline).

Every tensor is a pure function of (seed, tensor name, element index):

    key  = mix64(seed * GOLDEN + fnv1a64(name))
    bits = mix64(key + (i + 1) * GOLDEN)            # splitmix64 finaliser
    u    = (float(bits >> 40) - 2**23) * 2**-23      # exact fp32, uniform in [-1, 1)
    val  = fp32(fp32(u * scale) + offset)            # two IEEE ops, no fma
    bf16 = round-to-nearest-even(val)                # for bf16 tensors

The same function is implemented by the HIP kernel `zmi_fill_uniform` (csrc/zmi_misc.hip),
so a 3.2 GB model can be materialised on the GPU and a tiny one in numpy with
bit-identical values. Uniform noise with scale a has std a/sqrt(3).

Key names follow the reference `Zonos.state_dict()` (reference `zonos/model.py:22-51`,
`zonos/backbone/_torch.py:52-152`) and transformers' `DacModel` (`modeling_dac.py`).
"""
from __future__ import annotations

import math
from typing import Iterator

import numpy as np

from .config import EMB_VOCAB, HEAD_VOCAB, N_CODEBOOKS, ZonosConfig

GOLDEN = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1
SQRT3 = math.sqrt(3.0)


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & _M64
    return h


def mix64(z: int) -> int:
    z &= _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def tensor_key(seed: int, name: str) -> int:
    return mix64((seed * GOLDEN + fnv1a64(name)) & _M64)


def _mix64_np(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniform_f32(key: int, n: int, scale: float, offset: float = 0.0, start: int = 0) -> np.ndarray:
    """fp32 values of elements [start, start+n) of the stream `key` (see module doc)."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(key) + idx * np.uint64(GOLDEN)
        bits = _mix64_np(z)
    u24 = (bits >> np.uint64(40)).astype(np.float32)
    u = (u24 - np.float32(8388608.0)) * np.float32(1.0 / 8388608.0)
    v = u * np.float32(scale)
    if offset != 0.0:
        v = v + np.float32(offset)
    return v.astype(np.float32)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16 bit patterns (uint16)."""
    u = x.astype(np.float32).view(np.uint32)
    r = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << np.uint32(16)).view(np.float32)


# --------------------------------------------------------------------------------------
# Tensor inventory with init rules
# --------------------------------------------------------------------------------------
class Spec:
    """One synthetic tensor: name, shape, dtype ('bf16'|'f32'), uniform scale, offset."""

    __slots__ = ("name", "shape", "dtype", "scale", "offset")

    def __init__(self, name, shape, dtype, scale, offset=0.0):
        self.name, self.shape, self.dtype = name, tuple(int(s) for s in shape), dtype
        self.scale, self.offset = float(scale), float(offset)

    @property
    def numel(self) -> int:
        return int(np.prod(self.shape))


W_STD = 0.02


def zonos_specs(cfg: ZonosConfig) -> list[Spec]:
    """bf16 tensors of the Zonos model (un-padded reference shapes)."""
    bb = cfg.backbone
    if bb.is_hybrid:
        return hybrid_specs(cfg)
    d, hd = bb.d_model, bb.head_dim
    a = W_STD * SQRT3
    qkv = (bb.num_heads + 2 * bb.num_heads_kv) * hd
    ff = bb.attn_mlp_d_intermediate
    out = []
    for k in range(N_CODEBOOKS):
        out.append(Spec(f"embeddings.{k}.weight", (EMB_VOCAB, d), "bf16", a))
    for i in range(bb.n_layer):
        p = f"backbone.layers.{i}."
        out += [
            Spec(p + "norm.weight", (d,), "bf16", 0.1, 1.0),
            Spec(p + "norm.bias", (d,), "bf16", 0.02),
            Spec(p + "mixer.in_proj.weight", (qkv, d), "bf16", a),
            Spec(p + "mixer.out_proj.weight", (d, bb.num_heads * hd), "bf16", a),
            Spec(p + "norm2.weight", (d,), "bf16", 0.1, 1.0),
            Spec(p + "norm2.bias", (d,), "bf16", 0.02),
            Spec(p + "mlp.fc1.weight", (2 * ff, d), "bf16", a),
            Spec(p + "mlp.fc2.weight", (d, ff), "bf16", a),
        ]
    out += [Spec("backbone.norm_f.weight", (d,), "bf16", 0.1, 1.0),
            Spec("backbone.norm_f.bias", (d,), "bf16", 0.02)]
    for k in range(N_CODEBOOKS):
        out.append(Spec(f"heads.{k}.weight", (HEAD_VOCAB, d), "bf16", a))
    return out


def hybrid_specs(cfg: ZonosConfig) -> list[Spec]:
    """bf16 tensors of the hybrid model, mamba-ssm parameter names (Block: norm, mixer, norm2, mlp;
    Mamba2: in_proj, conv1d, dt_bias, A_log, D, norm, out_proj; MHA: in_proj, out_proj; GatedMLP: fc1,
    fc2). Init ranges follow Mamba2's: A = -exp(A_log) in [-16, -1]; dt = softplus(dt_bias + ..) around
    0.05-0.3 so the state carries several steps; D near 1."""
    bb = cfg.backbone
    d, a = bb.d_model, W_STD * SQRT3
    md = bb.mamba2_dims()
    out = [Spec(f"embeddings.{k}.weight", (EMB_VOCAB, d), "bf16", a) for k in range(N_CODEBOOKS)]
    for i in range(bb.n_layer):
        p = f"backbone.layers.{i}."
        out += [Spec(p + "norm.weight", (d,), "bf16", 0.1, 1.0), Spec(p + "norm.bias", (d,), "bf16", 0.02)]
        if i in bb.attn_layer_idx:
            hd = bb.head_dim
            out += [Spec(p + "mixer.in_proj.weight", ((bb.num_heads + 2 * bb.num_heads_kv) * hd, d), "bf16", a),
                    Spec(p + "mixer.out_proj.weight", (d, bb.num_heads * hd), "bf16", a)]
            ff = bb.attn_mlp_d_intermediate
        else:
            out += [Spec(p + "mixer.in_proj.weight", (md["d_in_proj"], d), "bf16", a),
                    Spec(p + "mixer.conv1d.weight", (md["conv_dim"], 1, md["d_conv"]), "bf16", 0.5),
                    Spec(p + "mixer.conv1d.bias", (md["conv_dim"],), "bf16", 0.1),
                    Spec(p + "mixer.dt_bias", (md["nheads"],), "bf16", 1.0, -2.0),
                    Spec(p + "mixer.A_log", (md["nheads"],), "bf16", 1.386, 1.386),
                    Spec(p + "mixer.D", (md["nheads"],), "bf16", 0.1, 1.0),
                    Spec(p + "mixer.norm.weight", (md["d_ssm"],), "bf16", 0.1, 1.0),
                    Spec(p + "mixer.out_proj.weight", (d, md["d_ssm"]), "bf16", W_STD * SQRT3)]
            ff = bb.d_intermediate
        if ff:
            out += [Spec(p + "norm2.weight", (d,), "bf16", 0.1, 1.0), Spec(p + "norm2.bias", (d,), "bf16", 0.02),
                    Spec(p + "mlp.fc1.weight", (2 * ff, d), "bf16", a), Spec(p + "mlp.fc2.weight", (d, ff), "bf16", a)]
    out += [Spec("backbone.norm_f.weight", (d,), "bf16", 0.1, 1.0),
            Spec("backbone.norm_f.bias", (d,), "bf16", 0.02)]
    out += [Spec(f"heads.{k}.weight", (HEAD_VOCAB, d), "bf16", a) for k in range(N_CODEBOOKS)]
    return out


# DAC 44.1 kHz decoder geometry (transformers DacConfig defaults)
DAC_LATENT = 1024          # encoder_hidden_size * 2**4
DAC_DEC_HIDDEN = 1536
DAC_STRIDES = (8, 8, 4, 2)
DAC_CODEBOOK_DIM = 8
DAC_DILATIONS = (1, 3, 9)


def dac_block_channels() -> list[tuple[int, int, int]]:
    """(c_in, c_out, stride) of the 4 decoder blocks: 1536->768->384->192->96."""
    out, c = [], DAC_DEC_HIDDEN
    for s in DAC_STRIDES:
        out.append((c, c // 2, s))
        c //= 2
    return out


def dac_specs() -> list[Spec]:
    """fp32 tensors of the DAC decoder path (quantizer.from_codes + decoder)."""
    out = []
    for i in range(N_CODEBOOKS):
        p = f"quantizer.quantizers.{i}."
        out += [Spec(p + "codebook.weight", (1024, DAC_CODEBOOK_DIM), "f32", SQRT3),
                Spec(p + "out_proj.weight", (DAC_LATENT, DAC_CODEBOOK_DIM, 1), "f32", 1 / math.sqrt(8)),
                Spec(p + "out_proj.bias", (DAC_LATENT,), "f32", 0.1)]

    def conv(name, cout, cin, k):
        bound = 1.0 / math.sqrt(cin * k)
        return [Spec(name + ".weight", (cout, cin, k), "f32", bound), Spec(name + ".bias", (cout,), "f32", bound)]

    def snake(name, c):
        return [Spec(name + ".alpha", (1, c, 1), "f32", 0.25, 1.0)]

    out += conv("decoder.conv1", DAC_DEC_HIDDEN, DAC_LATENT, 7)
    for j, (cin, cout, s) in enumerate(dac_block_channels()):
        p = f"decoder.block.{j}."
        out += snake(p + "snake1", cin)
        bound = 1.0 / math.sqrt(cout * 2 * s)
        out += [Spec(p + "conv_t1.weight", (cin, cout, 2 * s), "f32", bound),
                Spec(p + "conv_t1.bias", (cout,), "f32", bound)]
        for u in range(3):
            q = p + f"res_unit{u + 1}."
            out += snake(q + "snake1", cout) + conv(q + "conv1", cout, cout, 7)
            out += snake(q + "snake2", cout) + conv(q + "conv2", cout, cout, 1)
    c_last = dac_block_channels()[-1][1]
    out += snake("decoder.snake1", c_last) + conv("decoder.conv2", 1, c_last, 7)
    return out


DAC_ENC_HIDDEN = 64
DAC_ENC_STRIDES = (2, 4, 8, 8)


def dac_encoder_specs() -> list[Spec]:
    """fp32 tensors of the DAC encode path (encoder + quantizer in_proj), DacEncoder modeling_dac.py:444-475,
    DacEncoderBlock :212-234, DacVectorQuantize.in_proj :119."""
    out = []

    def conv(name, cout, cin, k):
        bound = 1.0 / math.sqrt(cin * k)
        return [Spec(name + ".weight", (cout, cin, k), "f32", bound), Spec(name + ".bias", (cout,), "f32", bound)]

    def snake(name, c):
        return [Spec(name + ".alpha", (1, c, 1), "f32", 0.25, 1.0)]

    out += conv("encoder.conv1", DAC_ENC_HIDDEN, 1, 7)
    c = DAC_ENC_HIDDEN
    for j, s in enumerate(DAC_ENC_STRIDES):
        p = f"encoder.block.{j}."
        for u in range(3):
            q = p + f"res_unit{u + 1}."
            out += snake(q + "snake1", c) + conv(q + "conv1", c, c, 7)
            out += snake(q + "snake2", c) + conv(q + "conv2", c, c, 1)
        out += snake(p + "snake1", c) + conv(p + "conv1", 2 * c, c, 2 * s)
        c *= 2
    out += snake("encoder.snake1", c) + conv("encoder.conv2", DAC_LATENT, c, 3)
    for i in range(N_CODEBOOKS):
        p = f"quantizer.quantizers.{i}."
        out += [Spec(p + "in_proj.weight", (DAC_CODEBOOK_DIM, DAC_LATENT, 1), "f32", 1 / math.sqrt(DAC_LATENT)),
                Spec(p + "in_proj.bias", (DAC_CODEBOOK_DIM,), "f32", 0.1)]
    return out


def prefix_conditioner_specs(conditioners: list[dict], d: int) -> list[Spec]:
    """bf16 parameters of a PrefixConditioner (reference state-dict names under `prefix_conditioner.`,
    conditioning.py:284-291), scaled like their module inits: embeddings and Fourier weights std 1,
    linear projections uniform(+-1/sqrt(fan_in)), learned uncond vectors small and nonzero, LayerNorm
    weight ~1."""
    from .conditioning import PrefixConditioner
    out = []
    for name, shape in PrefixConditioner(conditioners, d, "cpu").param_shapes().items():
        n = "prefix_conditioner." + name
        if name == "norm.weight":
            out.append(Spec(n, shape, "bf16", 0.1, 1.0))
        elif name.endswith("project.weight"):
            out.append(Spec(n, shape, "bf16", 1.0 / float(np.sqrt(shape[1]))))
        elif name == "norm.bias" or name.endswith("project.bias"):
            out.append(Spec(n, shape, "bf16", 0.02))
        elif name.endswith("uncond_vector"):
            out.append(Spec(n, shape, "bf16", 0.5))
        else:  # phoneme / integer embedders, Fourier weights
            out.append(Spec(n, shape, "bf16", SQRT3))
    return out


def synthetic_speaker_np(seed: int, dim: int = 128) -> np.ndarray:
    """[1, dim] bf16 bits: a speaker embedding for the speaker conditioner (std 0.5)."""
    key = tensor_key(seed, f"speaker/{dim}")
    return f32_to_bf16_bits(uniform_f32(key, dim, 0.5 * SQRT3)).reshape(1, dim)


def materialize_np(spec: Spec, seed: int = 0) -> np.ndarray:
    """numpy array for `spec` (bf16 returned as uint16 bit patterns)."""
    key = tensor_key(seed, spec.name)
    n = spec.numel
    chunks = []
    step = 1 << 24
    for s in range(0, n, step):
        chunks.append(uniform_f32(key, min(step, n - s), spec.scale, spec.offset, start=s))
    v = np.concatenate(chunks) if len(chunks) != 1 else chunks[0]
    if spec.dtype == "bf16":
        return f32_to_bf16_bits(v).reshape(spec.shape)
    return v.reshape(spec.shape)


def iter_torch_cpu(specs: list[Spec], seed: int = 0) -> Iterator[tuple[str, "torch.Tensor"]]:
    import torch
    for sp in specs:
        a = materialize_np(sp, seed)
        if sp.dtype == "bf16":
            t = torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
        else:
            t = torch.from_numpy(a.copy())
        yield sp.name, t


def synthetic_conditioning_np(seed: int, rows: int, length: int, d: int) -> np.ndarray:
    """[rows, length, d] bf16 bits: N(0,1)-scaled uniform prefix conditioning."""
    key = tensor_key(seed, f"prefix_conditioning/{rows}x{length}x{d}")
    return f32_to_bf16_bits(uniform_f32(key, rows * length * d, SQRT3)).reshape(rows, length, d)
