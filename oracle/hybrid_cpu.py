"""ORACLE — CPU restatement of the hybrid (Mamba2 + attention) backbone. TEST INFRASTRUCTURE ONLY.

PARITY UNPINNED. The reference's hybrid backbone (zonos/backbone/_mamba_ssm.py:9-57) is assembled
from three third-party packages the reference does not vendor and this image does not have:
mamba-ssm 2.2.4, causal-conv1d 1.5.0.post8 and flash-attn 2.7.4.post1 (pins: reference uv.lock,
SURVEY.md §2/§8c). No golden vector or reference output exists for it. This module restates their
published algorithms, operation for operation where the rounding points matter:

  Block.forward, fused_add_norm   mamba_ssm/modules/block.py + ops/triton/layer_norm.py layer_norm_fn:
                                  s = hidden + residual in fp32, residual_out = s in the residual dtype
                                  (bf16: residual_in_fp32=False), LayerNorm statistics on the fp32 s
  MambaSSMZonosBackbone.forward   _mamba_ssm.py:44-57: the layers, then layer_norm_fn(norm_f) on hidden +
                                  residual (prenorm=False)
  Mamba2.forward (prefill)        mamba_ssm/modules/mamba2.py: in_proj, conv_state = last d_conv raw xBC
                                  inputs, causal_conv1d_fn(silu), mamba_chunk_scan_combined(D, dt_bias,
                                  dt_softplus) -> y (fp32 internally, bf16 out) + final state -> ssm_state
  Mamba2.step (decode)            causal_conv1d_update(silu) + selective_state_update (Triton kernel: fp32
                                  state update, bf16 store, readout from the fp32 state, + D x)
  RMSNormGated                    ops/triton/layernorm_gated.py, norm_before_gate=False: rmsnorm(y silu(z)) w
  MHA                             mamba_ssm/modules/mha.py: in_proj -> q | k | v, flash-attn RotaryEmbedding
                                  (non-interleaved halves, cos / sin cached in the activation dtype), KV cache,
                                  causal softmax attention (fp32 softmax) -> out_proj

The chunked SSD scan of the prefill is restated as its defining recurrence (h_t = exp(dt_t A) h_{t-1}
+ dt_t B_t x_t, y_t = C_t h_t + D x_t, fp32); `ssd_chunked` below restates the chunked form
(mamba_ssm/modules/ssd_minimal.py ssd_minimal_discrete) and tests/test_hybrid_oracle.py checks that
the two agree, which is as far as the scan can be pinned without the package.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .zonos_cpu import OracleZonos


def add_layernorm(hidden, residual, w, b, eps):
    """layer_norm_fn(hidden, w, b, residual, prenorm=True): (normed bf16, residual_out bf16).
    residual=None: the first block (residual = hidden)."""
    s = hidden.float() if residual is None else hidden.float() + residual.float()
    res = s.to(torch.bfloat16)
    mean = s.mean(-1, keepdim=True)
    var = ((s - mean) ** 2).mean(-1, keepdim=True)
    rstd = 1.0 / torch.sqrt(var + eps)
    y = ((s - mean) * rstd) * w.float() + b.float()
    return y.to(torch.bfloat16), res


def gated_rmsnorm(y, z, w, eps=1e-5):
    """RMSNormGated(norm_before_gate=False, group_size = d_ssm) -> bf16."""
    zf = z.float()
    g = y.float() * (zf * torch.sigmoid(zf))
    rstd = 1.0 / torch.sqrt((g * g).mean(-1, keepdim=True) + eps)
    return ((g * rstd) * w.float()).to(torch.bfloat16)


def causal_conv_silu(window, w, b):
    """causal_conv1d: bias first, taps oldest first (fp32), SiLU, bf16. window [..., C, 4] raw inputs."""
    acc = b.float().expand(window.shape[:-1]).clone()
    for k in range(window.shape[-1]):
        acc = acc + w[:, k].float() * window[..., k].float()
    return (acc / (1.0 + torch.exp(-acc))).to(torch.bfloat16)


def softplus20(x):
    return torch.where(x <= 20.0, torch.log1p(torch.exp(x)), x)


def ssd_chunked(x, dt, A, B, C, chunk: int):
    """ssd_minimal_discrete (mamba_ssm/modules/ssd_minimal.py) in fp64: the chunked SSD form of the scan.
    x [b, l, h, p], dt [b, l, h], A [h], B / C [b, l, n] (one group). Returns y [b, l, h, p], final state."""
    b, l, h, p = x.shape
    n = B.shape[-1]
    X = (x * dt[..., None]).double()
    Adt = (A[None, None, :] * dt).double()                      # [b, l, h]
    nc = (l + chunk - 1) // chunk
    pad = nc * chunk - l
    if pad:
        X = F.pad(X, (0, 0, 0, 0, 0, pad))
        Adt = F.pad(Adt, (0, 0, 0, pad))
        B = F.pad(B, (0, 0, 0, pad))
        C = F.pad(C, (0, 0, 0, pad))
    X = X.view(b, nc, chunk, h, p)
    Adt = Adt.view(b, nc, chunk, h).permute(0, 3, 1, 2)         # [b, h, c, l]
    Bc = B.double().view(b, nc, chunk, n)
    Cc = C.double().view(b, nc, chunk, n)
    Acum = torch.cumsum(Adt, dim=-1)

    def segsum(a):
        t = a.size(-1)
        a = a[..., None].repeat(*([1] * a.dim()), t)
        mask = torch.tril(torch.ones(t, t, dtype=torch.bool), diagonal=-1)
        a = a.masked_fill(~mask, 0)
        s = torch.cumsum(a, dim=-2)
        return s.masked_fill(~torch.tril(torch.ones(t, t, dtype=torch.bool), diagonal=0), -torch.inf)

    L = torch.exp(segsum(Adt))                                   # [b, h, c, l, s]
    Y_diag = torch.einsum("bcln,bcsn,bhcls,bcshp->bclhp", Cc, Bc, L, X)
    decay_states = torch.exp(Acum[:, :, :, -1:] - Acum)
    states = torch.einsum("bcln,bhcl,bclhp->bchpn", Bc, decay_states, X)
    states = torch.cat([torch.zeros_like(states[:, :1]), states], dim=1)
    decay_chunk = torch.exp(segsum(F.pad(Acum[:, :, :, -1], (1, 0))))
    new_states = torch.einsum("bhzc,bchpn->bzhpn", decay_chunk, states)
    states, final = new_states[:, :-1], new_states[:, -1]
    Y_off = torch.einsum("bcln,bchpn,bhcl->bclhp", Cc, states, torch.exp(Acum))
    y = (Y_diag + Y_off).reshape(b, nc * chunk, h, p)[:, :l]
    return y, final


def ssd_recurrence(x, dt, A, B, C, state=None):
    """The defining recurrence, fp32 (what mamba2_scan computes). Returns y (no D term), final state."""
    b, l, h, p = x.shape
    n = B.shape[-1]
    st = torch.zeros(b, h, p, n) if state is None else state.float().clone()
    ys = []
    for t in range(l):
        dA = torch.exp(dt[:, t] * A[None, :])                                        # [b, h]
        dBx = (B[:, t, None, None, :] * dt[:, t, :, None, None]) * x[:, t, :, :, None]  # [b, h, p, n]
        st = st * dA[:, :, None, None] + dBx
        ys.append((st * C[:, t, None, None, :]).sum(-1))
    return torch.stack(ys, dim=1), st


def mamba2_step_ref(zx, window, ssm, cw, cb, dt_bias, A, D, md):
    """Mamba2.step after in_proj for b rows: zx [b, d_in_proj] bf16, window [b, conv_dim, d_conv] raw xBC
    inputs oldest first (the last one is this token's), ssm [b, h, p, n] bf16. Returns y = C.h + D x (bf16,
    before the gated norm) and the new bf16 state (causal_conv1d_update + selective_state_update)."""
    b = zx.shape[0]
    d_ssm, ds, nh, hd = md["d_ssm"], md["d_state"], md["nheads"], md["headdim"]
    dt = zx[:, 2 * d_ssm + 2 * ds:]
    xc = causal_conv_silu(window, cw, cb)
    x, B, C = xc.split([d_ssm, ds, ds], dim=-1)
    dtv = softplus20(dt.float() + dt_bias.float())
    dA = torch.exp(A[None, :] * dtv)
    xh = x.float().view(b, nh, hd)
    st = ssm.float() * dA[:, :, None, None] + (B[:, None, None, :].float() * dtv[:, :, None, None]) * xh[..., None]
    y = (st * C[:, None, None, :].float()).sum(-1) + xh * D[None, :, None]
    return y.to(torch.bfloat16).reshape(b, d_ssm), st.to(torch.bfloat16)


def mamba2_scan_ref(zx, cw, cb, dt_bias, A, D, md):
    """Mamba2.forward after in_proj from an empty cache: zx [b, s, d_in_proj] bf16. Returns y (bf16, before
    the gated norm), the final bf16 state and conv_state [b, conv_dim, d_conv] (the last raw inputs)."""
    b, s, _ = zx.shape
    d_ssm, ds, nh, hd, dc = md["d_ssm"], md["d_state"], md["nheads"], md["headdim"], md["d_conv"]
    xbc, dt = zx[..., d_ssm:2 * d_ssm + 2 * ds], zx[..., 2 * d_ssm + 2 * ds:]
    raw = xbc.transpose(1, 2)
    conv_state = F.pad(raw, (dc - s, 0))[..., -dc:] if s < dc else raw[..., -dc:]
    win = F.pad(raw, (dc - 1, 0)).unfold(-1, dc, 1)
    xc = causal_conv_silu(win.transpose(1, 2), cw, cb)
    x, B, C = xc.split([d_ssm, ds, ds], dim=-1)
    dtv = softplus20(dt.float() + dt_bias.float())
    xh = x.float().view(b, s, nh, hd)
    y, st = ssd_recurrence(xh, dtv, A, B.float(), C.float())
    y = (y + xh * D[None, None, :, None]).to(torch.bfloat16).reshape(b, s, d_ssm)
    return y, st.to(torch.bfloat16), conv_state.contiguous()


def rope_neox_tables(n_pos: int, dim: int, base: float = 10000.0):
    """flash_attn RotaryEmbedding._update_cos_sin_cache: fp32 angles, cos / sin cast to bf16."""
    inv = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.float32) / dim))
    ang = torch.outer(torch.arange(n_pos, dtype=torch.float32), inv)
    return torch.cos(ang).to(torch.bfloat16), torch.sin(ang).to(torch.bfloat16)


def apply_rope_neox(x, cos, sin):
    """apply_rotary (non-interleaved): x [..., hd] bf16, cos / sin [..., hd / 2] bf16; fp32 math, bf16 out."""
    half = x.shape[-1] // 2
    x0, x1 = x[..., :half].float(), x[..., half:].float()
    c, s = cos.float(), sin.float()
    return torch.cat([x0 * c - x1 * s, x0 * s + x1 * c], dim=-1).to(torch.bfloat16)


class OracleHybrid(OracleZonos):
    """CPU restatement of Zonos with the hybrid backbone (generate / heads / sampler from OracleZonos)."""

    def __init__(self, cfg, weights: dict):
        super().__init__(cfg, weights)
        bb = cfg.backbone
        self.md = bb.mamba2_dims()
        self.attn_idx = list(bb.attn_layer_idx)
        self.cos, self.sin = rope_neox_tables(16384, self.hd)

    def new_cache(self, rows: int, max_seqlen: int):
        md = self.md
        smax = max_seqlen if max_seqlen % 8 == 0 else max_seqlen + 8 - max_seqlen % 8
        c = {"offset": 0, "lengths": torch.zeros(rows, dtype=torch.int32), "kv": {}, "conv": {}, "ssm": {}}
        for i in range(self.n_layer):
            if i in self.attn_idx:
                c["kv"][i] = torch.zeros(rows, smax, 2, self.hkv, self.hd, dtype=torch.bfloat16)
            else:
                c["conv"][i] = torch.zeros(rows, md["conv_dim"], md["d_conv"], dtype=torch.bfloat16)
                c["ssm"][i] = torch.zeros(rows, md["nheads"], md["headdim"], md["d_state"], dtype=torch.bfloat16)
        return c

    # ---------------------------------------------------------------- mixers
    def _mamba(self, i, u, cache):
        md, w = self.md, self.w
        p = f"backbone.layers.{i}.mixer."
        b, s, _ = u.shape
        d_ssm, ds, nh, hd = md["d_ssm"], md["d_state"], md["nheads"], md["headdim"]
        zx = F.linear(u, w[p + "in_proj.weight"])
        z = zx[..., :d_ssm]
        cw, cb = w[p + "conv1d.weight"][:, 0, :], w[p + "conv1d.bias"]
        A = -torch.exp(w[p + "A_log"].float())
        D, dtb = w[p + "D"].float(), w[p + "dt_bias"].float()
        conv, ssm = cache["conv"][i], cache["ssm"][i]
        if cache["offset"] > 0:  # Mamba2.step
            assert s == 1
            win = torch.cat([conv[:b, :, 1:], zx[:, 0, d_ssm:2 * d_ssm + 2 * ds, None]], dim=-1)
            conv[:b] = win
            y, ssm[:b] = mamba2_step_ref(zx[:, 0], win, ssm[:b], cw, cb, dtb, A, D, md)
            y = y.view(b, 1, d_ssm)
        else:  # Mamba2.forward from an empty cache
            y, ssm[:b], conv[:b] = mamba2_scan_ref(zx, cw, cb, dtb, A, D, md)
        yn = gated_rmsnorm(y, z, w[p + "norm.weight"])
        return F.linear(yn, w[p + "out_proj.weight"])

    def _mha(self, i, u, cache):
        p = f"backbone.layers.{i}.mixer."
        b, s, _ = u.shape
        qs, ks = self.h * self.hd, self.hkv * self.hd
        q, k, v = F.linear(u, self.w[p + "in_proj.weight"]).split([qs, ks, ks], dim=-1)
        o0 = cache["offset"]
        pos = torch.arange(o0, o0 + s)
        cos, sin = self.cos[pos][None, :, None, :], self.sin[pos][None, :, None, :]
        q = apply_rope_neox(q.view(b, s, self.h, self.hd), cos, sin)
        k = apply_rope_neox(k.view(b, s, self.hkv, self.hd), cos, sin)
        kv = cache["kv"][i]
        kv[:b, o0:o0 + s, 0] = k
        kv[:b, o0:o0 + s, 1] = v.view(b, s, self.hkv, self.hd)
        kk, vv = kv[:b, :o0 + s].unbind(dim=-3)
        g = self.h // self.hkv
        qf = q.float().transpose(1, 2)                                                     # [b, h, s, hd]
        kf = kk.float().transpose(1, 2).repeat_interleave(g, dim=1)
        vf = vv.float().transpose(1, 2).repeat_interleave(g, dim=1)
        sc = qf @ kf.transpose(-1, -2) / (self.hd ** 0.5)
        mask = torch.arange(o0 + s)[None, :] > (torch.arange(s)[:, None] + o0)
        sc = sc.masked_fill(mask, -torch.inf)
        y = (torch.softmax(sc, dim=-1) @ vf).to(torch.bfloat16)
        y = y.transpose(1, 2).reshape(b, s, qs)
        return F.linear(y, self.w[p + "out_proj.weight"])

    def _gated_mlp(self, i, x):
        p = f"backbone.layers.{i}.mlp."
        y, gate = F.linear(x, self.w[p + "fc1.weight"]).chunk(2, dim=-1)
        return F.linear(y * F.silu(gate), self.w[p + "fc2.weight"])

    def backbone(self, h: torch.Tensor, cache) -> torch.Tensor:
        """_mamba_ssm.py:44-57 with mamba-ssm Block.forward (fused_add_norm, prenorm)."""
        bb, w = self.cfg.backbone, self.w
        hidden, residual = h, None
        for i in range(self.n_layer):
            pf = f"backbone.layers.{i}."
            x, residual = add_layernorm(hidden, residual, w[pf + "norm.weight"], w[pf + "norm.bias"], self.eps)
            if i in self.attn_idx:
                hidden = self._mha(i, x, cache)
                ff = bb.attn_mlp_d_intermediate
            else:
                hidden = self._mamba(i, x, cache)
                ff = bb.d_intermediate
            if ff:
                x, residual = add_layernorm(hidden, residual, w[pf + "norm2.weight"], w[pf + "norm2.bias"], self.eps)
                hidden = self._gated_mlp(i, x)
        out, _ = add_layernorm(hidden, residual, w["backbone.norm_f.weight"], w["backbone.norm_f.bias"], self.eps)
        return out
