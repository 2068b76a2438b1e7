"""HybridEngine: the Zonos-v0.1-hybrid backbone (Mamba2 + attention) on the HIP kernels.

Reference: zonos/backbone/_mamba_ssm.py:9-57 (MambaSSMZonosBackbone), whose blocks come from
mamba-ssm 2.2.4's create_block (absent here: parity unpinned, oracle/hybrid_cpu.py). Everything
around the backbone — delay pattern, prefill orchestration, heads, CFG, sampler, EOS state machine,
hipGraph-captured decode loop, slots — is HipEngine's; this class only swaps the layer plan:

  every block    layer_norm_fn prenorm (residual += hidden in fp32, LayerNorm): decode as the ADDLN
                 prologue of the block's first GEMV, prefill as zmi_add_layernorm (same arithmetic)
  Mamba2 block   zmi_mamba_block: in_proj GEMV + the Mamba2 step (conv ring + SiLU + selective state
                 update) in one launch, granule hand-off (zmi_mamba2_step as its own launch above 16 rows)
                 -> out_proj GEMV with the GRMS prologue (RMSNormGated; prefill: zmi_gated_rmsnorm and
                 zmi_mamba2_scan_ws over the sequence)
  MHA block      QKV GEMV (non-interleaved rotary as interleaved pairs on permuted q / k rows, bf16
                 cos / sin as flash-attn caches them) -> attention kernel -> out_proj GEMV
  optional MLP   (add + LayerNorm) fc1 SwiGLU GEMV -> fc2 GEMV       (d_intermediate > 0)
  norm_f         (add + LayerNorm) heads GEMV

State per slot row: the conv ring bf16 [4][conv_dim] and the SSM state bf16 [nheads][64][128] of
every Mamba2 layer (1.06 MB per row and layer at the Zonos-v0.1-hybrid dims), K / V of the attention
layers only.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .config import EMB_VOCAB, HEAD_VOCAB, N_CODEBOOKS, ROPE_TABLE_LEN
from .engine import HEADS_N, HEADS_N_PAD, HipEngine


def rope_table_neox(hd: int, n: int = ROPE_TABLE_LEN) -> torch.Tensor:
    """flash-attn RotaryEmbedding cache (mamba_ssm MHA, rotary_emb_dim = head dim): fp32 angles, cos / sin
    cast to bf16 (the activation dtype), stored as fp32 (cos, sin) pairs for the QKV epilogue."""
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2, dtype=torch.float32) / hd))
    ang = torch.outer(torch.arange(n, dtype=torch.float32), inv)
    return torch.stack([torch.cos(ang).bfloat16().float(), torch.sin(ang).bfloat16().float()], dim=-1).contiguous()


def neox_pair_perm(hd: int) -> torch.Tensor:
    """Row order putting element j next to j + hd/2 (the halves the non-interleaved rotary pairs), so the
    interleaved-pair RoPE epilogue applies it. q and k both carry it, so q.k is unchanged."""
    j = torch.arange(hd // 2)
    return torch.stack([j, j + hd // 2], dim=1).flatten()


class HybridEngine(HipEngine):
    hybrid = True

    prefill_batch = False  # the Mamba2 prefill scan takes one (cond, uncond) pair of sequences per pass

    def __init__(self, cfg, device="cuda", max_slots: int = 1, max_seqlen: int = 2048, max_prefill: int = 512):
        bb = cfg.backbone
        if bb.rms_norm or bb.residual_in_fp32:
            raise NotImplementedError("hybrid blocks are built for LayerNorm with bf16 residuals (Zonos-v0.1-hybrid)")
        self.md = bb.mamba2_dims()
        md = self.md
        if (md["headdim"], md["d_state"], md["d_conv"], md["ngroups"]) != (64, 128, 4, 1) or not md["rmsnorm"] \
                or md["norm_before_gate"] or md["D_has_hdim"]:
            raise NotImplementedError(f"Mamba2 geometry not built: {md}")
        # MHA / Mamba2 options the kernels do not implement must not load silently (mamba_ssm MHA defaults:
        # qkv_proj_bias / out_proj_bias True, causal False, rotary_emb_dim 0; Mamba2: dt_limit (0, inf))
        ac, sc = dict(bb.attn_cfg), dict(bb.ssm_cfg)
        hd = bb.d_model // int(ac.get("num_heads", 1))
        bad = [k for k, ok in (
            ("attn_cfg.rotary_emb_dim", int(ac.get("rotary_emb_dim", 0)) == hd),
            ("attn_cfg.rotary_emb_interleaved", not ac.get("rotary_emb_interleaved", False)),
            ("attn_cfg.rotary_emb_base", float(ac.get("rotary_emb_base", 10000.0)) == 10000.0),
            ("attn_cfg.qkv_proj_bias", not ac.get("qkv_proj_bias", True)),
            ("attn_cfg.out_proj_bias", not ac.get("out_proj_bias", True)),
            ("attn_cfg.causal", bool(ac.get("causal", False))),
            ("attn_cfg.softmax_scale", ac.get("softmax_scale") is None),
            ("attn_cfg.d_conv", int(ac.get("d_conv", 0)) == 0),
            ("attn_cfg.mlp_dim", int(ac.get("mlp_dim", 0)) == 0),
            ("ssm_cfg.dt_limit", tuple(float(v) for v in sc.get("dt_limit", (0.0, float("inf")))) == (0.0, float("inf"))),
            ("ssm_cfg.bias", not sc.get("bias", False)),
            ("ssm_cfg.conv_bias", bool(sc.get("conv_bias", True))),
            ("ssm_cfg.learnable_init_states", not sc.get("learnable_init_states", False)),
        ) if not ok]
        if bad:
            raise NotImplementedError(f"hybrid options not built by the HIP kernels: {bad}")
        self.attn_idx = sorted(int(i) for i in bb.attn_layer_idx)
        self.Fm = int(bb.d_intermediate)
        super().__init__(cfg, device, max_slots, max_seqlen, max_prefill)
        # the MHA blocks' QKV + attention as ONE launch (zmi_attn_block with the ADDLN projection prologue)
        self.attn_block = True
        # decode in_proj + Mamba2 step as ONE launch (zmi_mamba_block) for <= 16 rows at d_model 2048
        self.mamba_block = True
        # prefetch the layer's out_proj weights into the Infinity Cache during the step phase: measured slower
        # (C4 300 frames: 320 ms off; 321, 333 and 361 ms with 64, 192 and 32 prefetch workgroups), so off
        self.mamba_prefetch = False
        # the decode out_proj's RMSNormGated prologue reads g = y * gate written by the step (GRMS_G: 32 KB of activation
        # rows per workgroup at 2 rows) instead of y and the gate (GRMS: 48 KB); the same bits
        self.grms_g = True
        self.prefetch_blocks, self.prefetch_fc1_mb = 192, 0  # the MHA blocks' out_proj prefetch (measured in round 2)
        # the MHA blocks' out_proj inside the fused block (round 6; the prefetch above then stays off)
        self.attn_oproj_mha = True

    def _kv_layers(self) -> int:
        return len(self.attn_idx)

    def _alloc(self):
        super()._alloc()
        md, R, P, dev = self.md, self.R, self.max_prefill, self.dev
        nm = self.L - len(self.attn_idx)
        z = lambda *shape, dt=torch.bfloat16: torch.zeros(*shape, dtype=dt, device=dev)  # noqa: E731
        with torch.cuda.stream(self.stream):
            self.hid, self.nrm = z(R, self.d), z(R, self.d)
            self.x2 = z(R, self.d)  # the decode residual stream ping-pongs between self.x and self.x2
            self.zero_rows = z(R, self.d)  # block 0's "hidden": s = 0 + residual, exactly the residual
            self.zx, self.yb, self.yn = z(R, md["d_in_proj"]), z(R, md["d_ssm"]), z(R, md["d_ssm"])
            self.gz = z(R, md["d_ssm"], dt=torch.float32)  # decode: g = y * gate (grms_g) or the gate z * sigmoid(z)
            self.hid_pre, self.nrm_pre = z(2 * P, self.d), z(2 * P, self.d)
            self.zx_pre, self.yb_pre, self.yn_pre = z(2 * P, md["d_in_proj"]), z(2 * P, md["d_ssm"]), z(2 * P, md["d_ssm"])
            self.hm = z(R, max(self.Fm, self.F, 1))
            self.hm_pre = z(2 * P, max(self.Fm, self.F, 1))
            self.conv_ring = z(nm, R, md["d_conv"], md["conv_dim"])
            self.ssm = z(nm, R, md["nheads"], md["headdim"], md["d_state"])
            self.mgran = z(nm, R, md["d_in_proj"] // 2, dt=torch.int64)  # zmi_mamba_block hand-off granules
            ws = int(self.lib.zmi_mamba2_scan_ws_bytes(2 * P, md["d_ssm"], md["nheads"]))
            self.scan_ws = z(ws, dt=torch.uint8)  # zmi_mamba2_scan_ws: conv output, dt, dA of the prefill rows
            self.rope = rope_table_neox(self.hd).to(dev)
        self.stream.synchronize()

    # ------------------------------------------------------------------ weights
    def load_state_dict(self, sd: dict):
        """mamba-ssm parameter names (Block norm / mixer / norm2 / mlp; Mamba2, MHA, GatedMLP)."""
        bf = lambda t: t.to(self.dev, torch.bfloat16).contiguous()  # noqa: E731
        f32 = lambda t: t.to(self.dev, torch.bfloat16).float().contiguous()  # noqa: E731  (bf16 model params)
        md, hd = self.md, self.hd
        perm = neox_pair_perm(hd)
        with torch.cuda.stream(self.stream):
            w = {}
            if "embeddings.0.weight" in sd:
                w["emb"] = torch.stack([bf(sd[f"embeddings.{k}.weight"])[:EMB_VOCAB] for k in range(N_CODEBOOKS)])
            layers = []
            for i in range(self.L):
                p = f"backbone.layers.{i}."
                lw = dict(ln1_w=bf(sd[p + "norm.weight"]), ln1_b=bf(sd[p + "norm.bias"]))
                if i in self.attn_idx:
                    qkv = bf(sd[p + "mixer.in_proj.weight"])
                    nq, nk = self.H * hd, self.Hkv * hd
                    q = qkv[:nq].view(self.H, hd, -1)[:, perm.to(self.dev)].reshape(nq, -1)
                    k = qkv[nq:nq + nk].view(self.Hkv, hd, -1)[:, perm.to(self.dev)].reshape(nk, -1)
                    lw.update(kind="attn", kv=self.attn_idx.index(i),
                              qkv=self._pack(torch.cat([q, k, qkv[nq + nk:]]), nq + 2 * nk),
                              out=self._pack(sd[p + "mixer.out_proj.weight"], self.d))
                    ff = self.F
                else:
                    lw.update(kind="mamba", st=i - sum(1 for j in self.attn_idx if j < i),
                              in_proj=self._pack(sd[p + "mixer.in_proj.weight"], md["d_in_proj"]),
                              conv_w=bf(sd[p + "mixer.conv1d.weight"]).reshape(md["conv_dim"], md["d_conv"]).contiguous(),
                              conv_b=bf(sd[p + "mixer.conv1d.bias"]),
                              dt_bias=f32(sd[p + "mixer.dt_bias"]),
                              A=(-torch.exp(f32(sd[p + "mixer.A_log"]))).contiguous(),
                              D=f32(sd[p + "mixer.D"]),
                              norm_w=bf(sd[p + "mixer.norm.weight"]),
                              out=self._pack(sd[p + "mixer.out_proj.weight"], self.d))
                    ff = self.Fm
                if ff:
                    lw.update(ff=ff, ln2_w=bf(sd[p + "norm2.weight"]), ln2_b=bf(sd[p + "norm2.bias"]),
                              fc1=self._pack(sd[p + "mlp.fc1.weight"], 2 * ff, _lib.PACK_SWIGLU),
                              fc2=self._pack(sd[p + "mlp.fc2.weight"], self.d))
                layers.append(lw)
            w["layers"] = layers
            w["nf_w"], w["nf_b"] = bf(sd["backbone.norm_f.weight"]), bf(sd["backbone.norm_f.bias"])
            if "heads.0.weight" in sd:
                heads = torch.zeros(HEADS_N, self.d, dtype=torch.bfloat16, device=self.dev)
                for k in range(N_CODEBOOKS):
                    heads[k * 1026: k * 1026 + HEAD_VOCAB] = bf(sd[f"heads.{k}.weight"])[:HEAD_VOCAB]
                w["heads"] = self._pack(heads, HEADS_N_PAD)
                del heads
        self.stream.synchronize()
        self.w = w
        self._build_plan()

    def _reset_granules(self, slot: int):
        super()._reset_granules(slot)
        self.mgran[:, 2 * slot: 2 * slot + 2].zero_()

    # ------------------------------------------------------------------ launch helpers
    def _addln(self, hid, res, ln, out, m, store=True):
        lib, d, eps, s = self.lib, self.d, self.eps, self.sptr
        hp = None if hid is None else hid.data_ptr()
        rp, wp, bp, op = res.data_ptr(), ln[0].data_ptr(), ln[1].data_ptr(), out.data_ptr()
        st = 1 if store else 0

        def run():
            _lib.check(lib.zmi_add_layernorm(hp, d, rp, d, m, d, wp, bp, eps, op, d, st, s), "add_layernorm")
        return run

    def _mamba_args(self, lw, zx, y, m, row_pos, row_kv) -> _lib.Mamba2Args:
        md = self.md
        a = _lib.Mamba2Args()
        a.zxbcdt, a.ld_zx, a.M = zx.data_ptr(), md["d_in_proj"], m
        a.d_ssm, a.nheads, a.headdim, a.d_state, a.d_conv, a.ngroups = (md["d_ssm"], md["nheads"], md["headdim"],
                                                                        md["d_state"], md["d_conv"], md["ngroups"])
        a.conv_w, a.conv_b = lw["conv_w"].data_ptr(), lw["conv_b"].data_ptr()
        a.dt_bias, a.A, a.D = lw["dt_bias"].data_ptr(), lw["A"].data_ptr(), lw["D"].data_ptr()
        a.conv_ring, a.ssm = self.conv_ring[lw["st"]].data_ptr(), self.ssm[lw["st"]].data_ptr()
        a.y, a.ldy = y.data_ptr(), md["d_ssm"]
        a.row_pos = row_pos.data_ptr()
        a.row_kv = _lib.ptr(row_kv)
        return a

    def _gnorm(self, lw, y, zx, out, m):
        lib, md, s = self.lib, self.md, self.sptr
        yp, zp, wp, op = y.data_ptr(), zx.data_ptr(), lw["norm_w"].data_ptr(), out.data_ptr()

        def run():
            _lib.check(lib.zmi_gated_rmsnorm(yp, md["d_ssm"], zp, md["d_in_proj"], m, md["d_ssm"], wp, 1e-5, op,
                                             md["d_ssm"], s), "gated_rmsnorm")
        return run

    def _call_mamba_block(self, ia, sa, gran, out_w=None):
        lib, s, ep, gp = self.lib, self.sptr, self.blk_err[1:].data_ptr(), gran.data_ptr()  # word 1: the Mamba2 block
        ia.row_pos = sa.row_pos  # the in_proj epilogue tags its granules with the row's position + 1
        pf = _lib.Prefetch()
        if out_w is not None and self.prefetch_blocks > 0:  # out_proj's weights into the Infinity Cache
            pf.ptr[0], pf.bytes[0] = out_w.data_ptr(), out_w.numel() * 2
            pf.sink, pf.blocks = self.blk_err[2:].data_ptr(), self.prefetch_blocks

        def run():
            _lib.check(lib.zmi_mamba_block_pf(ctypes.byref(ia), ctypes.byref(sa), gp, ep, ctypes.byref(pf), s),
                       "mamba_block")
        run.args = (ia, sa)  # for tools (tools/hybrid_stamps.py sets ia.diag)
        return run

    def _call_step(self, a):
        lib, s = self.lib, self.sptr

        def run():
            _lib.check(lib.zmi_mamba2_step(ctypes.byref(a), s), "mamba2_step")
        return run

    def _layer_items(self, lw, m, x, hid, nrm, zx, yb, yn, hm, q, attn, row_kv, row_pos, first, seq_len=None,
                     max_pos=None):
        """Launches of one block over m rows (decode: seq_len None; prefill: sequences of seq_len rows)."""
        d, md, qd = self.d, self.md, self.H * self.hd
        items = [("call", self._addln(None if first else hid, x, (lw["ln1_w"], lw["ln1_b"]), nrm, m))]
        if lw["kind"] == "attn":
            j = lw["kv"]
            qkv_n = (self.H + 2 * self.Hkv) * self.hd
            items.append(("gemv", self._gemv(lw["qkv"], nrm, m, qkv_n, d, _lib.EPI_QKV, q, qd,
                                             kv=(self.kc[j], self.vc[j]), row_kv=row_kv, row_pos=row_pos)))
            if seq_len is None:
                items.append(("attn", j))
            else:
                items.append(("call", lambda j=j: self._attention(j, q, m, row_kv, row_pos, max_pos, attn)))
            items.append(("gemv", self._gemv(lw["out"], attn, m, d, qd, _lib.EPI_STORE, hid, d)))
        else:
            items.append(("gemv", self._gemv(lw["in_proj"], nrm, m, md["d_in_proj"], d, _lib.EPI_STORE, zx,
                                             md["d_in_proj"])))
            if seq_len is None:
                items.append(("call", self._call_step(self._mamba_args(lw, zx, yb, m, row_pos, None))))
            else:
                a = self._mamba_args(lw, zx, yb, m, row_pos, row_kv)
                lib, s, wp, wn = self.lib, self.sptr, self.scan_ws.data_ptr(), self.scan_ws.numel()
                items.append(("call", lambda a=a: _lib.check(lib.zmi_mamba2_scan_ws(ctypes.byref(a), seq_len, wp, wn,
                                                                                    s), "mamba2_scan_ws")))
            items.append(("call", self._gnorm(lw, yb, zx, yn, m)))
            items.append(("gemv", self._gemv(lw["out"], yn, m, d, md["d_ssm"], _lib.EPI_STORE, hid, d)))
        if lw.get("ff"):
            ff = lw["ff"]
            items.append(("call", self._addln(hid, x, (lw["ln2_w"], lw["ln2_b"]), nrm, m)))
            items.append(("gemv", self._gemv(lw["fc1"], nrm, m, 2 * ff, d, _lib.EPI_SWIGLU, hm, ff)))
            items.append(("gemv", self._gemv(lw["fc2"], hm, m, d, ff, _lib.EPI_STORE, hid, d)))
        return items

    # ------------------------------------------------------------------ decode plan
    def _fused(self, item, pro, aux, ld_aux, res_out=None):
        a, epi = item
        a.pro, a.aux, a.ld_aux, a.res_out = pro, aux.data_ptr(), ld_aux, _lib.ptr(res_out)
        return ("gemv", (a, epi))

    def _plan(self, rows: int, form: str = "none") -> list:
        """Decode launches. The block norms run as GEMV prologues: layer_norm_fn(hidden, residual) as ADDLN
        on the consuming GEMV (in_proj / qkv / fc1 / heads; the new residual goes to the other of two
        buffers, since the other workgroups still read the old one), RMSNormGated as GRMS on out_proj (up
        to 4 rows, the gate z * sigmoid(z) formed once per channel by the Mamba2 step kernel: the y and f32
        gate rows of a larger tile would not fit the LDS image). Same arithmetic as the
        prefill's standalone norm kernels."""
        if (rows, form) not in self._plans:
            w, d, md, qd = self.w, self.d, self.md, self.H * self.hd
            res = [self.x, self.x2]
            cur = 0
            plan = []

            def normed_gemv(item, ln, first):
                nonlocal cur
                item[0].ln_w, item[0].ln_b = ln[0].data_ptr(), ln[1].data_ptr()
                if first:  # block 0 (residual=None): hidden = 0, so s is the embedding and stays the residual
                    return self._fused(item, _lib.PRO_ADDLN, res[cur], d, None)
                out = self._fused(item, _lib.PRO_ADDLN, res[cur], d, res[1 - cur])
                cur = 1 - cur
                return out

            for i, lw in enumerate(w["layers"]):
                x_in = self.zero_rows if i == 0 else self.hid
                ln1 = (lw["ln1_w"], lw["ln1_b"])
                if lw["kind"] == "attn":
                    j = lw["kv"]
                    qkv_n = (self.H + 2 * self.Hkv) * self.hd
                    qkv = normed_gemv(self._gemv(lw["qkv"], x_in, rows, qkv_n, d, _lib.EPI_QKV, self.q, qd,
                                                 kv=(self.kc[j], self.vc[j]), row_kv=self.row_kv,
                                                 row_pos=self.row_pos), ln1, i == 0)
                    # out_proj as the fused block's fourth role (zmi_attn_block_oproj, plain store into the hidden rows)
                    oproj = (self._use_attn_block(rows, form) and self.attn_oproj_mha and form in ("split", "split24")
                             and qd == d)
                    if self._use_attn_block(rows, form):
                        pf = _lib.Prefetch()
                        if self.prefetch_blocks > 0 and not oproj:  # out_proj's weights into the Infinity Cache meanwhile
                            pf.ptr[0], pf.bytes[0] = lw["out"].data_ptr(), lw["out"].numel() * 2
                            pf.sink, pf.blocks = self.blk_err[2:].data_ptr(), self.prefetch_blocks
                        o_item = self._gemv(lw["out"], self.attn, rows, d, qd, _lib.EPI_STORE, self.hid, d)
                        plan.append(("attnblk", (qkv[1][0], j, pf, self._block_slices(form)) +
                                     ((o_item[0],) if oproj else ())))
                    else:
                        plan.append(qkv)
                        plan.append(("attn", j))
                    if not oproj:
                        plan.append(("gemv", self._gemv(lw["out"], self.attn, rows, d, qd, _lib.EPI_STORE, self.hid, d)))
                else:
                    inp = normed_gemv(self._gemv(lw["in_proj"], x_in, rows, md["d_in_proj"], d, _lib.EPI_STORE,
                                                 self.zx, md["d_in_proj"]), ln1, i == 0)
                    sa = self._mamba_args(lw, self.zx, self.yb, rows, self.row_pos, None)
                    fuse_g = rows <= 4  # the f32 gate rows of a larger tile would not fit the LDS image
                    if fuse_g:  # the step writes g = y * gate (gz_g), the out_proj's GRMS_G prologue reads only g
                        sa.gz, sa.gz_g = self.gz.data_ptr(), 1 if self.grms_g else 0
                    if self.mamba_block and d == 2048 and rows <= 16:
                        plan.append(("call", self._call_mamba_block(inp[1][0], sa, self.mgran[lw["st"]],
                                                                    lw["out"] if self.mamba_prefetch else None)))
                    else:
                        plan.append(inp)
                        plan.append(("call", self._call_step(sa)))
                    out = self._gemv(lw["out"], self.yb, rows, d, md["d_ssm"], _lib.EPI_STORE, self.hid, d)
                    if fuse_g:
                        out[0].ln_w = lw["norm_w"].data_ptr()
                        out[0].eps = 1e-5  # RMSNormGated's own eps (mamba2.py)
                        plan.append(self._fused(out, _lib.PRO_GRMS_G if self.grms_g else _lib.PRO_GRMS, self.gz,
                                                md["d_ssm"]))
                    else:
                        plan.append(("call", self._gnorm(lw, self.yb, self.zx, self.yn, rows)))
                        plan.append(("gemv", self._gemv(lw["out"], self.yn, rows, d, md["d_ssm"], _lib.EPI_STORE,
                                                        self.hid, d)))
                if lw.get("ff"):
                    ff = lw["ff"]
                    plan.append(normed_gemv(self._gemv(lw["fc1"], self.hid, rows, 2 * ff, d, _lib.EPI_SWIGLU, self.hm,
                                                       ff), (lw["ln2_w"], lw["ln2_b"]), False))
                    plan.append(("gemv", self._gemv(lw["fc2"], self.hm, rows, d, ff, _lib.EPI_STORE, self.hid, d)))
            heads = self._gemv(w["heads"], self.hid, rows, HEADS_N_PAD, d, _lib.EPI_LOGITS, self.logits, 0,
                               n_valid=HEADS_N)
            heads[0].ln_w, heads[0].ln_b = w["nf_w"].data_ptr(), w["nf_b"].data_ptr()
            plan.append(self._fused(heads, _lib.PRO_ADDLN, res[cur], d, None))
            self._plans[(rows, form)] = plan
        return self._plans[(rows, form)]

    # ------------------------------------------------------------------ prefill
    def _prefill_layers(self, m: int, max_pos: int):
        """m rows = sequences of max_pos + 1 rows each, every sequence from position 0 (Mamba2.forward
        from an empty cache; the reference's step() takes one token at a time after that)."""
        seq_len = max_pos + 1
        if m % seq_len:
            raise ValueError("hybrid prefill: rows must be whole sequences starting at position 0")
        for i, lw in enumerate(self.w["layers"]):
            for kind, item in self._layer_items(lw, m, self.x_pre, self.hid_pre, self.nrm_pre, self.zx_pre,
                                                self.yb_pre, self.yn_pre, self.hm_pre, self.q_pre, self.attn_pre,
                                                self.row_kv_pre, self.row_pos_pre, first=(i == 0), seq_len=seq_len,
                                                max_pos=max_pos):
                if kind == "gemv":
                    self._run_gemv(item)
                else:
                    item()

    def _prefill_logits(self, s_len: int):
        d = self.d
        off = (s_len - 1) * d * 2  # bytes: row s_len - 1, then the uncond row s_len further on
        lib = self.lib
        _lib.check(lib.zmi_add_layernorm(self.hid_pre.data_ptr() + off, s_len * d, self.x_pre.data_ptr() + off,
                                         s_len * d, 2, d, self.w["nf_w"].data_ptr(), self.w["nf_b"].data_ptr(),
                                         self.eps, self.x_last.data_ptr(), d, 0, self.sptr), "norm_f")
        self._run_gemv(self._gemv(self.w["heads"], self.x_last, 2, HEADS_N_PAD, d, _lib.EPI_LOGITS, self.logits_pre,
                                  0, n_valid=HEADS_N))

    def final_norm_pre(self, m: int, out: torch.Tensor):
        _lib.check(self.lib.zmi_add_layernorm(self.hid_pre.data_ptr(), self.d, self.x_pre.data_ptr(), self.d, m,
                                              self.d, self.w["nf_w"].data_ptr(), self.w["nf_b"].data_ptr(), self.eps,
                                              out.data_ptr(), self.d, 0, self.sptr), "norm_f")

    def inference_cache(self) -> dict:
        """{layer: (K, V^T)} for MHA layers, {layer: (conv ring, ssm state)} for Mamba2 layers."""
        out = {}
        for i, lw in enumerate(self.w["layers"]):
            if lw["kind"] == "attn":
                out[i] = (self.kc[lw["kv"]], self.vc[lw["kv"]])
            else:
                out[i] = (self.conv_ring[lw["st"]], self.ssm[lw["st"]])
        return out
