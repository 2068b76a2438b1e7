"""HipEngine: device state + launch plan of the Zonos transformer hot path on one MI355X.

Host-side orchestration in Python (PyTorch-ROCm is used only for device memory and the
stream); every device op goes through the C ABI of libzonos_hip.so. The decode step
(~5 launches per layer + embed + heads + sampler) is enqueued once under hipGraph capture
and replayed per step; all per-step state (positions, offsets, EOS state machine) lives on
the device, so a step needs no host synchronisation (reference zonos/model.py:276-307 syncs
the host several times per step).

Batch layout: utterance slot s owns activation / KV rows 2s (conditional) and 2s+1
(unconditional), i.e. the reference's `hidden_states.repeat(2, 1, 1)` CFG pair
(model.py:142) interleaved per slot. Each slot runs the reference's batch_size=1 semantics.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from . import synthetic as syn
from .config import EMB_VOCAB, HEAD_VOCAB, N_CODEBOOKS, ROPE_TABLE_LEN, ZonosConfig

HEADS_N = N_CODEBOOKS * 1026            # 9 heads x (1025 + 1 pad row), model.py:37 + utils.py:12-27
HEADS_N_PAD = (HEADS_N + 15) // 16 * 16
PREFILL_BATCH_ROWS = 2048  # rows of one batched prefill pass (prefill_many): 6 C2-sized utterances (2 x 161)
BLK_ROWS_MAX = 16  # rows zmi_attn_block takes (one MFMA row tile, include/zonos_hip.h)


def rope_table(hd: int, n: int = ROPE_TABLE_LEN) -> torch.Tensor:
    """(cos, sin) table in fp32 computed exactly as precompute_freqs_cis (_torch.py:9-15)."""
    inv = 1.0 / (10000.0 ** (torch.arange(0, hd, 2)[: hd // 2].float() / hd))
    ang = torch.outer(torch.arange(n, device=inv.device), inv)
    cis = torch.polar(torch.ones_like(ang), ang)
    return torch.stack([cis.real, cis.imag], dim=-1).contiguous()


_XCD_CHECKED = False


def _check_xcd_dealing(lib, sptr):
    """Set ZMI_OPT_XC_HANDOFF to write-through (1) unless this device deals workgroups round-robin over its XCDs."""
    global _XCD_CHECKED
    if _XCD_CHECKED:
        return
    ok = lib.zmi_xcd_dealing(sptr)
    if ok < 0:
        raise RuntimeError(f"zmi_xcd_dealing: {lib.zmi_last_error().decode()}")
    if ok == 0:
        _lib.check(lib.zmi_set_option(_lib.OPT_XC_HANDOFF, 1), "set_option")
    _XCD_CHECKED = True


@dataclass
class SamplingParams:
    """Reference `sample_from_logits` keywords (sampling.py:117-129) + CFG scale + seed."""
    temperature: float = 1.0
    top_p: float = 0.0
    top_k: int = 0
    min_p: float = 0.0
    linear: float = 0.0
    conf: float = 0.0
    quad: float = 0.0
    repetition_penalty: float = 3.0
    repetition_penalty_window: int = 2
    cfg_scale: float = 2.0
    seed: int = 0

    @classmethod
    def from_dict(cls, d: dict, cfg_scale: float, seed: int) -> "SamplingParams":
        known = {"temperature", "top_p", "top_k", "min_p", "linear", "conf", "quad", "repetition_penalty",
                 "repetition_penalty_window"}
        bad = set(d) - known
        if bad:
            raise TypeError(f"sample_from_logits() got unexpected keyword argument(s) {sorted(bad)}")
        return cls(**d, cfg_scale=float(cfg_scale), seed=int(seed))

    def to_c(self) -> _lib.Sampling:
        return _lib.Sampling(self.temperature, self.top_p, self.min_p, self.linear, self.conf, self.quad,
                             self.repetition_penalty, self.cfg_scale, int(self.top_k),
                             int(self.repetition_penalty_window), self.seed & ((1 << 64) - 1))


def _round8(n: int) -> int:
    return n if n % 8 == 0 else n + 8 - n % 8


class HipEngine:
    hybrid = False
    prefill_batch = True  # prefill_many packs several slots into one pass (the hybrid's scan does not)

    def __init__(self, cfg: ZonosConfig, device="cuda", max_slots: int = 1, max_seqlen: int = 2048,
                 max_prefill: int = 512):
        bb = cfg.backbone
        if bb.ssm_cfg and not self.hybrid:
            raise ValueError("hybrid (mamba-ssm) configs run on HybridEngine (make_engine picks it)")
        self.cfg = cfg
        self.dev = torch.device(device)
        self.d, self.L, self.H, self.Hkv = bb.d_model, bb.n_layer, bb.num_heads, bb.num_heads_kv
        self.hd = self.d // self.H
        self.F = bb.attn_mlp_d_intermediate
        self.eps = float(bb.norm_epsilon)
        if self.hd != 128:
            raise ValueError("the HIP attention kernels are built for head_dim 128")
        self.S = int(max_slots)
        self.R = 2 * self.S
        self.smax = min(_round8(int(max_seqlen)), ROPE_TABLE_LEN)
        self.tcap = self.smax  # delayed frames per slot never exceed KV positions
        self.max_prefill = int(max_prefill)
        # prefill rows one pass can hold: prefill_many() packs several slots' rows (2 x S each) into one pass
        # through the layers, so the weights stream once per batch of utterances instead of once per utterance
        self.pre_rows = max(2 * self.max_prefill, PREFILL_BATCH_ROWS if self.prefill_batch else 0)
        self.lib = _lib.lib()
        self.stream = torch.cuda.Stream(self.dev)
        self.sptr = self.stream.cuda_stream
        # the fused attention block hands chunk maxima and partials over through the XCD's L2 (ZMI_OPT_XC_HANDOFF 0),
        # which needs the round-robin workgroup dealing over the XCDs; checked once per process (a probe launch)
        _check_xcd_dealing(self.lib, self.sptr)
        self.w = None
        self.attn_variant = 0  # zmi_attention_variant kernel choice (0 = library; all give identical bits)
        # decode QKV + attention as ONE launch (zmi_attn_block) where it applies: <= `attn_block_rows` rows
        # and positions below the fused forms' reach; identical bits either way (speed only)
        self.attn_block = True
        self.attn_block_slices = 8
        # fused forms tried in order, each where every row's position is below its reach: "split" (one
        # workgroup per 128-key chunk, positions < 1024), "self" (every slice scores all keys, < 1024),
        # "split24" (24 chunk workgroups per (row, kv head), < 3072: batch-1 utterances up to the reference's
        # default 30 s), "xs" (slices exchange scores, < 1280); beyond, separate launches. The form is picked
        # per run of steps from host-side position bounds; all forms give identical bits. 30 s batch-1 line:
        # steps past position 1280 1167-1219 us with separate launches, 1073-1141 with "split24"; at 1161
        # "split24" 1078.5 against "xs" 1082-1086 (profiles/r04_split24_ab.jsonl)
        self.attn_forms = ("split", "split24", "xs")
        # the fused forms for <= `attn_block_rows` rows, "xs" and "split24" for <= `attn_xs_rows`: C5-shaped steps (1000 frames
        # after a 590-position context) at 4 / 8 / 16 rows take 1.232 / 1.516 / 1.902 ms with the fused forms,
        # 1.267 / 1.554 / 1.730 with separate QKV + attention launches, 1.223 / 1.516 / 1.80 without "xs"
        # (profiles/r03_attn_block_rows_ab.jsonl)
        self.attn_block_rows = 8
        self.attn_xs_rows = 2
        self.attn_self_slices = 8
        # prefetch-only workgroups in that launch warm the Infinity Cache with out_proj's weights and the
        # first `prefetch_fc1_mb` MB of fc1's while the attention runs (speed only). With out_proj and fc1 as
        # separate launches: C2 step 971 us (192 blocks, out_proj only), 959 (192, + 8 MB of fc1), 944-947
        # (256, + 4-8 MB), 966 (256, + 16 MB), 974 (512, + 8 MB) (profiles/r03_prefetch_ab.jsonl)
        # round 6, after the hand-offs through L2: 128 workgroups x 8 MB 896.6-899.2 us, 256 x 8 MB 905, 64 / 96 x 8 MB 903 /
        # 905, 128 x 6 / 12 / 16 MB 903 / 906 / 919 (profiles/r06_prefetch_sizing_ab.jsonl)
        self.prefetch_blocks = 128
        self.prefetch_fc1_mb = 8
        # the same prefetch role in the separate chunked attention launch (steps of > 8 rows, positions past the
        # fused forms' reach): workgroups at the end of its grid read out_proj's weights and the first
        # `attn_prefetch_fc1_mb` MB of fc1's while the chunks exchange maxima and merge (0 blocks = off). C5-shaped
        # job (8 slots, 2000 new frames): 1.776-1.786 ms per step without, 1.749 with 128 workgroups, 1.760-1.765
        # with 256 (+ 16 MB of fc1: 1.764); C3 sample unchanged (profiles/r04_attn_prefetch_ab.jsonl). Round 5, with
        # the block-form attention: C3 share 133.39-133.41x with 256 against 132.97-133.06 (128) and 133.15-133.24
        # (384), C5-shaped job 1.702-1.708 ms either way (profiles/r05_attn_prefetch_c3_c5_ab.jsonl)
        self.attn_prefetch_blocks = 256
        self.attn_prefetch_fc1_mb = 8
        # what the second range is: "fc1" (its head) or "qkv" (the next layer's QKV weights, the heads' on the
        # last layer: they would have to survive out_proj + fc1 + fc2 in the Infinity Cache)
        self.prefetch_second = "fc1"
        # out_proj inside the chunk-split fused block (zmi_attn_block_oproj): extra workgroups load its weights
        # during the attention chain and gather the attention output from the merging workgroups' granules, so
        # no out_proj launch follows (identical bits; the prefetch role then warms only fc1's head)
        self.attn_oproj = True
        # ... also in the 24-chunk form (batch-1 steps at positions 1024 .. 3071)
        self.attn_oproj_wide = True
        self.heads_groups = 0  # column groups of the heads GEMV (0: the library's choice)
        self.fc1_groups = 0  # column groups of the decode fc1 GEMV (0: the library's choice, 2)
        # fc2 (K = 8192) over >= `splitk_rows` rows and out_proj (K = 2048) over >= `splitk_o_rows` rows as
        # split-K GEMMs (zmi_gemv_splitk: each column block reads the activation rows once, and the reduce can
        # write the next LayerNorm; identical bits); 0 = never. out_proj split-K: C5-shaped 16-row step 1.732 vs
        # 1.741 ms, C3 sample 151.3 vs 149.5x (profiles/r03_splitk_oproj2_ab.jsonl)
        self.splitk_rows = 16
        self.splitk_o_rows = 16
        # the hybrid's Mamba2 out_proj (K = d_ssm = 4096, EPI_STORE) over >= `splitk_m_rows` rows (its prefill: the
        # GEMV form re-read every row's 8 KB activation row per 8-column group, 67 us at 322 rows)
        self.splitk_m_rows = 16
        # decode steps whose slots all sample greedily use the one-workgroup-per-slot sampler
        # (zmi_sample_step_greedy: identical results, no in-launch hand-off between codebooks)
        self.greedy_sampler = True
        # decode steps per hipGraph replay (a run of k steps replays the graph of graph_steps steps k // graph_steps
        # times, then the one-step graph for the rest; the same launches in the same order). C2 step at position
        # 591: 950.2-950.5 us with 1, 946.8 with 4, 945.8-946.0 with 8, 945.2 with 16 (profiles/r05_graph_steps_ab.jsonl)
        self.graph_steps = 16
        self.graph_steps_max_slots = 8
        # generate_batch steps only slots 0 .. the highest busy one (bucketed), not every slot
        self.batch_shrink = True
        self.slot_greedy = [False] * self.S
        self._plans: dict[tuple, list] = {}
        self._graphs: dict[tuple, int] = {}
        # host-side upper bound of each slot's next decode position (prefill sets it, every step adds 1):
        # it picks the attention form of a run of steps without reading the device
        self.pos_hi = [0] * self.S
        self.n_kv = self._kv_layers()
        self._alloc()

    def _kv_layers(self) -> int:
        """Layers with a KV cache (every layer of the transformer)."""
        return self.L

    # ------------------------------------------------------------------ allocation
    def _alloc(self):
        d, R, S, dev = self.d, self.R, self.S, self.dev
        qd = self.H * self.hd
        z = lambda *shape, dt=torch.bfloat16: torch.zeros(*shape, dtype=dt, device=dev)  # noqa: E731
        with torch.cuda.stream(self.stream):
            self.x, self.q, self.attn = z(R, d), z(R, qd), z(R, qd)
            self.xn = z(R, d)  # LayerNorm'd rows of a many-slot decode step (pre-pass, > 16 rows)
            self.h = z(R, self.F)
            self.logits = z(R, N_CODEBOOKS, 1026, dt=torch.float32)
            self.row_kv = z(R, dt=torch.int32)
            self.row_pos = torch.full((R,), -1, dtype=torch.int32, device=dev)  # every row inactive
            self.kc = z(self.n_kv, R, self.Hkv, self.smax, self.hd)   # K  [layer][row][kv head][position][hd]
            self.vc = z(self.n_kv, R, self.Hkv, self.hd, self.smax)   # V^T [layer][row][kv head][hd][position]
            nq = max(R, self.pre_rows)
            wb = self.lib.zmi_attention_work_bytes(nq, self.H, self.Hkv, self.hd, self.smax - 1)
            if wb < 0:
                raise ValueError("attention geometry not supported by the HIP kernel")
            self.attn_work = z(wb, dt=torch.uint8)  # first word: hand-off timeout flag
            nf = self.lib.zmi_attention_partial_floats(nq, self.H, self.Hkv, self.hd, self.smax - 1)
            self.attn_o = z(nf, dt=torch.float32)        # attention chunk partials (zmi_attn_merge.h)
            self.attn_lm = z(nf // self.hd * 2, dt=torch.float32)
            # zmi_attn_block hand-off granules {value, tag = position + 1}, one area per layer and row; a row's
            # areas are zeroed when it starts an utterance (prefill), and its error word. Only the first
            # BLK_ROWS_MAX rows can run the fused block (one 16-row tile), so only they get an area: at 128 rows
            # (C3's 64 slots) 26 x 16 areas of 104 KB instead of 26 x 128
            self.blk_rows = min(R, BLK_ROWS_MAX)
            self.blk_gran = z(self.n_kv, self.blk_rows, self.lib.zmi_attn_block_gran_words(1, self.Hkv),
                              dt=torch.int64)
            self.blk_err = z(4, dt=torch.int32)  # [0] attn_block, [1] mamba_block, [2] prefetch sink
            # zmi_gemv_splitk's fp32 segment sums (fc2 / out_proj over many rows: decode and prefill)
            self.splitk_part = z(self.lib.zmi_gemv_splitk_floats(max(R, self.pre_rows), d), dt=torch.float32)
            self.samp_cnt = z(S, dt=torch.int32)
            self.next_tok = z(S, N_CODEBOOKS, dt=torch.int32)
            self.st = {k: z(S, dt=torch.int32) for k in
                       ("active", "pos", "offset", "remaining", "stopping", "step", "total_len")}
            self.delayed = torch.full((S, N_CODEBOOKS, self.tcap), 1025, dtype=torch.int32, device=dev)
            self.params = z(S * ctypes.sizeof(_lib.Sampling), dt=torch.uint8)
            P2 = self.pre_rows
            self.x_pre, self.q_pre, self.attn_pre = z(P2, d), z(P2, qd), z(P2, qd)
            self.xn_pre = z(P2, d)  # LayerNorm'd prefill rows
            self.h_pre = z(P2, self.F)
            self.row_kv_pre = z(P2, dt=torch.int32)
            self.row_pos_pre = z(P2, dt=torch.int32)
            self.x_last = z(2, d)
            self.logits_pre = z(2, N_CODEBOOKS, 1026, dt=torch.float32)
            self.rope = rope_table(self.hd).to(dev)
        self.slots = _lib.Slots(*(self.st[k].data_ptr() for k in ("active", "pos", "offset", "remaining",
                                                                      "stopping", "step")),
                                self.delayed.data_ptr(), self.params.data_ptr(), self.st["total_len"].data_ptr(),
                                self.tcap, S)
        self.stream.synchronize()

    # ------------------------------------------------------------------ weights
    def _pack(self, w: torch.Tensor, n_pad: int, mode: int = _lib.PACK_IDENTITY) -> torch.Tensor:
        w = w.to(self.dev, torch.bfloat16).contiguous()
        n_src, k = w.shape
        out = torch.empty(n_pad * k, dtype=torch.bfloat16, device=self.dev)
        _lib.check(self.lib.zmi_pack_weight(w.data_ptr(), out.data_ptr(), n_src, k, n_pad, mode, self.sptr), "pack")
        return out

    def load_state_dict(self, sd: dict):
        """Reference state_dict names (model.py:22-51, _torch.py:52-152); heads [1025, d] or [1026, d]."""
        bf = lambda t: t.to(self.dev, torch.bfloat16).contiguous()  # noqa: E731
        with torch.cuda.stream(self.stream):
            w = {}
            if "embeddings.0.weight" in sd:  # absent for a backbone-only load (backbone.py)
                w["emb"] = torch.stack([bf(sd[f"embeddings.{k}.weight"])[:EMB_VOCAB] for k in range(N_CODEBOOKS)])
            qkv_n = (self.H + 2 * self.Hkv) * self.hd
            layers = []
            for i in range(self.L):
                p = f"backbone.layers.{i}."
                layers.append(dict(
                    ln1_w=bf(sd[p + "norm.weight"]), ln1_b=bf(sd[p + "norm.bias"]),
                    qkv=self._pack(sd[p + "mixer.in_proj.weight"], qkv_n),
                    out=self._pack(sd[p + "mixer.out_proj.weight"], self.d),
                    ln2_w=bf(sd[p + "norm2.weight"]), ln2_b=bf(sd[p + "norm2.bias"]),
                    fc1=self._pack(sd[p + "mlp.fc1.weight"], 2 * self.F, _lib.PACK_SWIGLU),
                    fc2=self._pack(sd[p + "mlp.fc2.weight"], self.d)))
            w["layers"] = layers
            w["nf_w"], w["nf_b"] = bf(sd["backbone.norm_f.weight"]), bf(sd["backbone.norm_f.bias"])
            if "heads.0.weight" in sd:
                heads = torch.zeros(HEADS_N, self.d, dtype=torch.bfloat16, device=self.dev)
                for k in range(N_CODEBOOKS):
                    hw = bf(sd[f"heads.{k}.weight"])[:HEAD_VOCAB]
                    heads[k * 1026: k * 1026 + HEAD_VOCAB] = hw
                w["heads"] = self._pack(heads, HEADS_N_PAD)
                del heads
        self.stream.synchronize()
        self.w = w
        self._build_plan()

    def init_synthetic(self, seed: int = 0, zero_eos: bool = False, eos_row_scale: float | None = None):
        """Materialise the synthetic weights of synthetic.zonos_specs on the GPU (bit-identical to numpy)."""
        sd = {}
        with torch.cuda.stream(self.stream):
            for sp in syn.zonos_specs(self.cfg):
                t = torch.empty(sp.shape, dtype=torch.bfloat16, device=self.dev)
                _lib.check(self.lib.zmi_fill_uniform(t.data_ptr(), sp.numel, syn.tensor_key(seed, sp.name),
                                                     sp.scale, sp.offset, 0, self.sptr), "fill")
                sd[sp.name] = t
            h0 = sd["heads.0.weight"]
            if zero_eos:
                h0[1024] = 0
            if eos_row_scale is not None:
                h0[1024] = (h0[1024].float() * eos_row_scale).to(torch.bfloat16)
        self.load_state_dict(sd)

    # ------------------------------------------------------------------ launch plan
    def _gemv(self, W, X, M, N, K, epi, out, ldo, n_valid=None, ln=None, kv=None, row_kv=None, row_pos=None):
        a = _lib.GemvArgs()
        a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
        if ln is not None:
            a.ln_w, a.ln_b = ln[0].data_ptr(), ln[1].data_ptr()
        a.eps = self.eps
        a.out, a.ldo = out.data_ptr(), ldo
        a.n_valid = N if n_valid is None else n_valid
        if kv is not None:
            a.row_kv, a.row_pos = row_kv.data_ptr(), row_pos.data_ptr()
            a.k_cache, a.v_cache = kv[0].data_ptr(), kv[1].data_ptr()
            a.smax, a.hq, a.hkv, a.hd = self.smax, self.H, self.Hkv, self.hd
            a.rope = self.rope.data_ptr()
        return (a, epi)

    def _run_gemv(self, item):
        a, epi = item
        if self._use_splitk(a, epi):
            _lib.check(self.lib.zmi_gemv_splitk(ctypes.byref(a), epi, self.splitk_part.data_ptr(),
                                                self.splitk_part.numel(), self.sptr), "gemv_splitk")
            return
        _lib.check(self.lib.zmi_gemv_launch(ctypes.byref(a), epi, self.sptr), "gemv")

    def _use_splitk(self, a, epi) -> bool:
        lo = {8192: self.splitk_rows, 2048: self.splitk_o_rows, 4096: self.splitk_m_rows}.get(a.K, 0)
        want = _lib.EPI_STORE if a.K == 4096 else _lib.EPI_RESIDUAL  # 4096: the hybrid's Mamba2 out_proj (d_ssm)
        return (lo > 0 and a.M >= lo and epi == want and not a.ln_w and a.pro == _lib.PRO_AUTO
                and a.N % 64 == 0 and a.n_valid == a.N
                and a.M * a.N * (8 if a.K == 8192 else 4) <= self.splitk_part.numel())

    def _build_plan(self):
        """Invalidate the per-row-count decode plans and graphs (new weights or buffers)."""
        for g in self._graphs.values():
            _lib.check(self.lib.zmi_graph_destroy(g))
        self._graphs.clear()
        self._plans.clear()

    def _block_slices(self, form: str) -> int:
        """zmi_attn_block `slices` argument of a fused form."""
        if form == "split":
            return 8 | _lib.ATTNBLK_SPLIT
        if form == "split24":  # 24 chunk workgroups per (row, kv head): positions < 3072
            return 24 | _lib.ATTNBLK_SPLIT
        return self.attn_self_slices | _lib.ATTNBLK_SELF if form == "self" else self.attn_block_slices

    def _forms(self, rows: int) -> list:
        """(form, last position it accepts) of the fused decode block, fastest first; "none" = separate
        QKV and attention launches (any position)."""
        out = []
        if (self.attn_block and rows <= min(self.attn_block_rows, self.blk_rows) and self.d == 2048
                and self.H == 4 * self.Hkv):
            for f in self.attn_forms:
                if f not in ("xs", "split24") or rows <= self.attn_xs_rows:
                    out.append((f, self.lib.zmi_attn_block_max_pos(self._block_slices(f))))
        return out + [("none", 1 << 30)]

    def _use_attn_block(self, rows: int, form: str | None = None) -> bool:
        return form != "none" and any(f == form for f, _ in self._forms(rows))

    def _segments(self, n: int, slots: int) -> list:
        """Split a run of n decode steps of slots 0..slots-1 into (steps, form) pieces: each piece's
        positions (host bound pos_hi .. + steps - 1) stay within its form's reach."""
        rows = 2 * slots
        p0 = max(self.pos_hi[:slots])
        segs = []
        while n > 0:
            for form, last in self._forms(rows):
                if p0 <= last:
                    k = min(n, last - p0 + 1)
                    break
            if segs and segs[-1][1] == form:
                segs[-1] = (segs[-1][0] + k, form)
            else:
                segs.append((k, form))
            n -= k
            p0 += k
        return segs

    def _plan(self, rows: int, form: str = "none") -> list:
        """Decode-step launches for the first `rows` rows (slots 0 .. rows/2 - 1). Every kernel's
        per-row arithmetic is independent of `rows` and of the launch form, so a slot decodes
        identically in any plan."""
        if (rows, form) not in self._plans:
            w, d, qd = self.w, self.d, self.H * self.hd
            qkv_n = (self.H + 2 * self.Hkv) * self.hd
            fused = self._use_attn_block(rows, form)
            # past a few rows every column-block workgroup's LayerNorm of all of them costs more than the
            # launch that normalises them once per layer (fc1 at 16 rows: 30.7 us with the prologue);
            # zmi_layernorm_rows gives the prologue's bits, so the plan may switch at any row count
            pre = rows > 4
            plan = []
            ln_ready = [False]  # the previous split-K fc2 already wrote the LayerNorm'd rows to xn

            def normed(ln):
                """(activation rows, prologue LayerNorm) of a LayerNorm'd GEMV, with the pre-pass item."""
                if not pre:
                    return self.x, ln
                if ln_ready[0]:
                    ln_ready[0] = False
                    return self.xn, None
                plan.append(("call", lambda ln=ln: _lib.check(self.lib.zmi_layernorm_rows(
                    self.x.data_ptr(), d, rows, d, ln[0].data_ptr(), ln[1].data_ptr(), self.eps, self.xn.data_ptr(),
                    d, self.sptr), "ln")))
                return self.xn, None

            for i, lw in enumerate(w["layers"]):
                kv = (self.kc[i], self.vc[i])
                xin, ln = normed((lw["ln1_w"], lw["ln1_b"])) if not fused else (self.x, (lw["ln1_w"], lw["ln1_b"]))
                qkv = self._gemv(lw["qkv"], xin, rows, qkv_n, d, _lib.EPI_QKV, self.q, qd,
                                 ln=ln, kv=kv, row_kv=self.row_kv, row_pos=self.row_pos)
                oproj = fused and self._use_attn_oproj(form)
                if fused:
                    pf = _lib.Prefetch()
                    if self.prefetch_blocks > 0:
                        if not oproj:  # (the fused out_proj role loads its weights itself)
                            pf.ptr[0], pf.bytes[0] = lw["out"].data_ptr(), lw["out"].numel() * 2
                        if self.prefetch_second == "qkv":
                            nw = w["heads"] if i + 1 == len(w["layers"]) else w["layers"][i + 1]["qkv"]
                        else:
                            nw = lw["fc1"]
                        pf.ptr[1] = nw.data_ptr()
                        pf.bytes[1] = min(nw.numel() * 2, int(self.prefetch_fc1_mb * 2 ** 20))
                        pf.sink, pf.blocks = self.blk_err[2:].data_ptr(), self.prefetch_blocks
                    o_fused = self._gemv(lw["out"], self.attn, rows, d, qd, _lib.EPI_RESIDUAL, self.x, d)[0] if oproj else None
                    plan.append(("attnblk", (qkv[0], i, pf, self._block_slices(form), o_fused)))
                else:
                    plan.append(("gemv", qkv))
                    apf = None
                    if self.attn_prefetch_blocks > 0:
                        apf = _lib.Prefetch()
                        apf.ptr[0], apf.bytes[0] = lw["out"].data_ptr(), lw["out"].numel() * 2
                        apf.ptr[1] = lw["fc1"].data_ptr()
                        apf.bytes[1] = min(lw["fc1"].numel() * 2, int(self.attn_prefetch_fc1_mb * 2 ** 20))
                        apf.sink, apf.blocks = self.blk_err[2:].data_ptr(), self.attn_prefetch_blocks
                    plan.append(("attn", (i, apf)))
                o_item = self._gemv(lw["out"], self.attn, rows, d, qd, _lib.EPI_RESIDUAL, self.x, d)
                if oproj:  # out_proj ran inside the fused block
                    xin, ln = normed((lw["ln2_w"], lw["ln2_b"]))
                    f1 = self._gemv(lw["fc1"], xin, rows, 2 * self.F, d, _lib.EPI_SWIGLU, self.h, self.F, ln=ln)
                    f1[0].groups = self.fc1_groups
                    plan.append(("gemv", f1))
                else:
                    if pre and self._use_splitk(*o_item) and d == 2048:
                        # the split-K reduce also writes LayerNorm(new x) for fc1 (no pre-pass launch)
                        plan.append(("splitkln", (o_item, (lw["ln2_w"], lw["ln2_b"]))))
                        ln_ready[0] = True
                    else:
                        plan.append(("gemv", o_item))
                    xin, ln = normed((lw["ln2_w"], lw["ln2_b"]))
                    plan.append(("gemv", self._gemv(lw["fc1"], xin, rows, 2 * self.F, d, _lib.EPI_SWIGLU, self.h,
                                                    self.F, ln=ln)))
                fc2 = self._gemv(lw["fc2"], self.h, rows, d, self.F, _lib.EPI_RESIDUAL, self.x, d)
                last = i + 1 == len(w["layers"])
                nxt = (w["nf_w"], w["nf_b"]) if last else (w["layers"][i + 1]["ln1_w"], w["layers"][i + 1]["ln1_b"])
                if pre and (last or not fused) and self._use_splitk(*fc2) and d == 2048:
                    # the split-K reduce also writes LayerNorm(new x) for the next op (no pre-pass launch)
                    plan.append(("splitkln", (fc2, nxt)))
                    ln_ready[0] = True
                else:
                    plan.append(("gemv", fc2))
            xin, ln = normed((w["nf_w"], w["nf_b"]))
            heads = self._gemv(w["heads"], xin, rows, HEADS_N_PAD, d, _lib.EPI_LOGITS, self.logits, 0,
                               n_valid=HEADS_N, ln=ln)
            heads[0].groups = self.heads_groups
            plan.append(("gemv", heads))
            self._plans[(rows, form)] = plan
        return self._plans[(rows, form)]

    def _attention(self, i, q, n_query, row_kv, row_pos, max_pos, out, pf=None):
        _lib.check(self.lib.zmi_attention_pf(
            q.data_ptr(), self.H * self.hd, self.kc[i].data_ptr(), self.vc[i].data_ptr(), _lib.ptr(row_kv),
            row_pos.data_ptr(), n_query, self.H, self.Hkv, self.hd, self.smax, max_pos, out.data_ptr(), self.H * self.hd,
            self.attn_o.data_ptr(), self.attn_lm.data_ptr(), self.attn_work.data_ptr(), self.attn_variant,
            None if pf is None else ctypes.byref(pf), self.sptr), "attention")

    def _run_attn_block(self, item):
        a, i, pf, slices = item[:4]
        o = item[4] if len(item) > 4 else None
        if o is not None:
            _lib.check(self.lib.zmi_attn_block_oproj(ctypes.byref(a), ctypes.byref(o), self.blk_gran[i].data_ptr(),
                                                     self.blk_err.data_ptr(), self.attn.data_ptr(), self.H * self.hd,
                                                     slices, ctypes.byref(pf), self.sptr), "attn_block_oproj")
            return
        _lib.check(self.lib.zmi_attn_block_pf(ctypes.byref(a), self.blk_gran[i].data_ptr(), self.blk_err.data_ptr(),
                                              self.attn.data_ptr(), self.H * self.hd, slices,
                                              ctypes.byref(pf), self.sptr), "attn_block")

    def _use_attn_oproj(self, form: str) -> bool:
        """out_proj inside the fused block: the chunk-split forms (8 and 24 chunks) of a LayerNorm'd transformer block."""
        wide_ok = form == "split24" and self.attn_oproj_wide
        return self.attn_oproj and (form == "split" or wide_ok) and not self.hybrid and self.H * self.hd == self.d

    def check_errors(self):
        """Raise if a launch gave up waiting on an in-launch hand-off (bounded spin) or refused a row past
        its reach. The flags are cleared first, so a later utterance (after a fresh prefill) runs clean."""
        attn = int(self.attn_work[:4].view(torch.int32).item())
        blk, mamba = (int(v) for v in self.blk_err[:2].tolist())
        if attn or blk or mamba:
            with torch.cuda.stream(self.stream):  # ordered with the engine's launches
                self.attn_work[:4].zero_()
                self.blk_err[:2].zero_()
            self.stream.synchronize()
        if attn:
            raise RuntimeError("attention: a cross-block hand-off timed out (results of that launch are invalid)")
        if blk:
            raise RuntimeError("attn_block: a hand-off wait timed out or a row was past the form's reach "
                               "(results are invalid)")
        if mamba:
            raise RuntimeError("mamba_block: a wait for the in_proj output timed out (results are invalid)")

    def refresh_inputs(self):
        """Recompute every slot's input embedding + row tables from the delayed codes (after a host-side
        edit of `delayed`, e.g. teacher forcing in tests); normally the sampler produces them."""
        _lib.check(self.lib.zmi_embed_step(ctypes.byref(self.slots), self.w["emb"].data_ptr(), self.d,
                                           self.x.data_ptr(), self.row_kv.data_ptr(), self.row_pos.data_ptr(),
                                           self.sptr), "embed")

    def _greedy_step(self, slot_begin: int, count: int) -> bool:
        return self.greedy_sampler and all(self.slot_greedy[slot_begin: slot_begin + count])

    def _sample(self, logits, noise, mode, slot_begin, count):
        if mode == 0 and noise is None and self._greedy_step(slot_begin, count):
            _lib.check(self.lib.zmi_sample_step_greedy(ctypes.byref(self.slots), logits.data_ptr(),
                                                       self.next_tok.data_ptr(), slot_begin, count,
                                                       self.w["emb"].data_ptr(), self.d, self.x.data_ptr(),
                                                       self.row_kv.data_ptr(), self.row_pos.data_ptr(), self.sptr),
                       "sample_greedy")
            return
        _lib.check(self.lib.zmi_sample_step(ctypes.byref(self.slots), logits.data_ptr(),
                                            None if noise is None else noise.data_ptr(), self.next_tok.data_ptr(),
                                            self.samp_cnt.data_ptr(), mode, slot_begin, count,
                                            self.w["emb"].data_ptr(), self.d, self.x.data_ptr(),
                                            self.row_kv.data_ptr(), self.row_pos.data_ptr(), self.sptr), "sample")

    def _rows(self, slots: int | None) -> int:
        s = self.S if slots is None else int(slots)
        if not 1 <= s <= self.S:
            raise ValueError(f"slots {s} outside 1..{self.S}")
        return 2 * s

    def enqueue_step(self, noise: torch.Tensor | None = None, slots: int | None = None, form: str | None = None):
        """One decode step for slots 0 .. slots-1 (default: all; reference model.py:276-307), enqueued
        on self.stream. The step's input embeddings and (kv row, position) tables were written by
        the previous sampler launch (or the prefill's), fused into its frame-write epilogue.
        form: the attention form (default: from the slots' position bounds; the bound advances)."""
        rows = self._rows(slots)
        if form is None:
            form = self._segments(1, rows // 2)[0][1]
            self._advance(1, rows // 2)
        for kind, item in self._plan(rows, form):
            if kind == "gemv":
                self._run_gemv(item)
            elif kind == "attnblk":
                self._run_attn_block(item)
            elif kind == "splitkln":
                (a, epi), ln = item
                _lib.check(self.lib.zmi_gemv_splitk_ln(ctypes.byref(a), epi, self.splitk_part.data_ptr(),
                                                       self.splitk_part.numel(), ln[0].data_ptr(), ln[1].data_ptr(),
                                                       self.eps, self.xn.data_ptr(), self.d, self.sptr), "gemv_splitk_ln")
            elif kind == "attn":
                # decode: query row r caches into KV row r, so no row table (kv_row = NULL)
                i, pf = item if isinstance(item, tuple) else (item, None)  # (layer, prefetch) or a KV layer index
                self._attention(i, self.q, rows, None, self.row_pos, self.smax - 1, self.attn, pf)
            else:  # "call": a prepared launch (hybrid kernels)
                item()
        self._sample(self.logits, noise, 0, 0, rows // 2)

    def capture(self, slots: int | None = None, form: str = "none", steps: int = 1):
        """The hipGraph of `steps` consecutive decode steps of slots 0 .. slots-1 in one attention form (the loop
        state lives on the device, so a graph of several steps is the one-step graph's launches repeated)."""
        rows = self._rows(slots)
        key = (rows, form, self._greedy_step(0, rows // 2), steps)
        if key not in self._graphs:
            _lib.check(self.lib.zmi_graph_begin(self.sptr), "graph_begin")
            try:
                for _ in range(steps):
                    self.enqueue_step(slots=rows // 2, form=form)
            finally:
                g = ctypes.c_void_p()
                _lib.check(self.lib.zmi_graph_end(self.sptr, ctypes.byref(g)), "graph_end")
            self._graphs[key] = g.value
        return self._graphs[key]

    def _advance(self, n: int, slots: int):
        for s in range(slots):
            self.pos_hi[s] += n

    def step(self, n: int = 1, use_graph: bool = True, slots: int | None = None):
        """n decode steps of slots 0 .. slots-1, as runs of hipGraph replays (one graph per attention
        form: a run switches form where the slots' position bound crosses a form's reach)."""
        if n <= 0:
            return
        s = self._rows(slots) // 2
        for k, form in self._segments(n, s):
            if use_graph:
                # multi-step graphs only for small batches: the many-slot share (C3) captures a graph per busy-slot
                # bucket inside its timed run, and there the 16-step captures cost more than the replay seams they
                # save (C3 share 133.9x with 1 step per graph against 132.5-132.7x with 16)
                u = self.graph_steps if s <= self.graph_steps_max_slots else 1
                if u > 1 and k >= u:  # runs of u-step graphs, then the remainder one step per replay
                    _lib.check(self.lib.zmi_graph_launch(self.capture(s, form, u), k // u, self.sptr), "graph_launch")
                if k % u or u <= 1:
                    _lib.check(self.lib.zmi_graph_launch(self.capture(s, form), k % u if u > 1 else k, self.sptr),
                               "graph_launch")
            else:
                for _ in range(k):
                    self.enqueue_step(slots=s, form=form)
            self._advance(k, s)

    # ------------------------------------------------------------------ prefill
    def _prefill_check(self, cond: torch.Tensor, prefix: torch.Tensor | None, max_new_tokens: int) -> int:
        lc = cond.shape[1]
        p = 0 if prefix is None else int(prefix.shape[-1])
        s_len = lc + p + 1
        if s_len > self.max_prefill:
            raise ValueError(f"prefill length {s_len} > engine max_prefill {self.max_prefill}")
        if s_len + max_new_tokens + 8 > self.smax or p + max_new_tokens + 9 > self.tcap:
            raise ValueError("utterance longer than the engine's KV capacity")
        if cond.shape[0] != 2 or cond.shape[2] != self.d:
            raise ValueError("prefix_conditioning must be [2 (cond, uncond), Lc, d_model]")
        return s_len

    def _prefill_stage(self, slot: int, cond: torch.Tensor, prefix: torch.Tensor | None, max_new_tokens: int,
                       params: SamplingParams, off: int, s_len: int):
        """The slot's sampling parameters, delayed-code buffer and granules, and its 2 x s_len prefill rows
        (cond, uncond) at row `off` of the prefill buffers (reference model.py:181-196, 240-250)."""
        assert 0 <= slot < self.S
        L, d = self.lib, self.d
        lc = cond.shape[1]
        p = s_len - lc - 1
        total = p + max_new_tokens + 9
        cond = cond.to(self.dev, torch.bfloat16)
        pr = torch.zeros(N_CODEBOOKS, max(p, 1), dtype=torch.int32, device=self.dev)
        if p:
            pr[:, :p] = prefix.reshape(N_CODEBOOKS, p).to(self.dev, torch.int32)
        cp = torch.tensor(bytearray(params.to_c()), dtype=torch.uint8)
        sz = ctypes.sizeof(_lib.Sampling)
        self.params[slot * sz:(slot + 1) * sz].copy_(cp)
        self.slot_greedy[slot] = params.temperature <= 0
        _lib.check(L.zmi_delay_init(ctypes.byref(self.slots), slot, pr.data_ptr(), p, total, self.sptr), "delay")
        self._reset_granules(slot)  # no granule of an earlier utterance may match a tag
        xp = self.x_pre[off: off + 2 * s_len]
        xp[:lc] = cond[0]
        xp[s_len: s_len + lc] = cond[1]
        codes = self.delayed[slot]
        for half in range(2):
            _lib.check(L.zmi_embed_codes(codes.data_ptr(), self.tcap, p + 1, self.w["emb"].data_ptr(), d,
                                         xp[half * s_len + lc].data_ptr(), d, self.sptr), "embed_codes")
        ar = torch.arange(s_len, dtype=torch.int32, device=self.dev)
        self.row_pos_pre[off: off + 2 * s_len] = torch.cat([ar, ar])
        self.row_kv_pre[off: off + s_len] = 2 * slot
        self.row_kv_pre[off + s_len: off + 2 * s_len] = 2 * slot + 1

    def _prefill_finish(self, slot: int, max_new_tokens: int, off: int, s_len: int, p: int, noise):
        """Heads of the slot's last prefill rows, slot state, first sample + frame write (model.py:251-264)."""
        self._prefill_logits(s_len) if off == 0 else self._prefill_logits(s_len, off)
        vals = {"active": 1, "pos": s_len, "offset": p, "remaining": max_new_tokens + 8, "stopping": 0,
                "step": 0, "total_len": p + max_new_tokens + 9}
        for k, v in vals.items():
            self.st[k][slot] = v
        self._sample(self.logits_pre, noise, 1, slot, 1)
        self.pos_hi[slot] = s_len

    def prefill(self, slot: int, cond: torch.Tensor, prefix: torch.Tensor | None, max_new_tokens: int,
                params: SamplingParams, noise: torch.Tensor | None = None):
        """_prefill + first sample + frame write (reference model.py:240-264) for one slot."""
        s_len = self._prefill_check(cond, prefix, max_new_tokens)
        p = s_len - cond.shape[1] - 1
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.stream):
            self._prefill_stage(slot, cond, prefix, max_new_tokens, params, 0, s_len)
            self._prefill_layers(2 * s_len, s_len - 1)
            self._prefill_finish(slot, max_new_tokens, 0, s_len, p, noise)
        return s_len

    def prefill_many(self, items) -> list:
        """prefill() of several slots: items are (slot, cond, prefix, max_new_tokens, params). Their rows are
        packed into passes of up to `pre_rows` rows, each pass through the layers once (one weight stream for
        all of them). Every kernel's per-row arithmetic is independent of the rows beside it (the GEMV / GEMM /
        split-K forms and the attention are tested batch-invariant), so each slot decodes exactly as if it had
        been prefilled alone (generate_batch == generate)."""
        items = list(items)
        if not self.prefill_batch or len(items) <= 1:
            return [self.prefill(*it) for it in items]
        lens = [self._prefill_check(it[1], it[2], it[3]) for it in items]
        groups, cur, rows = [], [], 0
        for it, s_len in zip(items, lens):
            if cur and rows + 2 * s_len > self.pre_rows:
                groups.append(cur)
                cur, rows = [], 0
            cur.append((it, s_len, rows))
            rows += 2 * s_len
        groups.append(cur)
        self.stream.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.stream):
            for g in groups:
                for (slot, cond, prefix, mnt, params), s_len, off in g:
                    self._prefill_stage(slot, cond, prefix, mnt, params, off, s_len)
                m = g[-1][2] + 2 * g[-1][1]
                self._prefill_layers(m, max(s_len for _, s_len, _ in g) - 1)
                for (slot, cond, prefix, mnt, params), s_len, off in g:
                    self._prefill_finish(slot, mnt, off, s_len, s_len - cond.shape[1] - 1, None)
        return lens

    def _reset_granules(self, slot: int):
        """Zero the in-launch hand-off granules of the slot's rows (tags are positions + 1)."""
        if 2 * slot < self.blk_rows:
            self.blk_gran[:, 2 * slot: 2 * slot + 2].zero_()

    def _prefill_logits(self, s_len: int, off: int = 0):
        """Heads of the last position of the cond / uncond prefill rows (starting at row `off`) -> logits_pre
        (model.py:103-116)."""
        xp = self.x_pre
        self.x_last[0] = xp[off + s_len - 1]
        self.x_last[1] = xp[off + 2 * s_len - 1]
        self._run_gemv(self._gemv(self.w["heads"], self.x_last, 2, HEADS_N_PAD, self.d, _lib.EPI_LOGITS,
                                  self.logits_pre, 0, n_valid=HEADS_N, ln=(self.w["nf_w"], self.w["nf_b"])))

    def final_norm_pre(self, m: int, out: torch.Tensor):
        """norm_f of the first m prefill rows into out (the backbone plugin's output)."""
        _lib.check(self.lib.zmi_layernorm_rows(self.x_pre.data_ptr(), self.d, m, self.d, self.w["nf_w"].data_ptr(),
                                               self.w["nf_b"].data_ptr(), self.eps, out.data_ptr(), self.d, self.sptr),
                   "norm_f")

    def _ln_pre(self, m: int, ln, out: torch.Tensor):
        """LayerNorm of the m prefill rows once per layer (zmi_layernorm_rows: the GEMV prologue's arithmetic,
        bit for bit), so the prefill GEMVs' many row-tile x column-block workgroups run without a prologue."""
        _lib.check(self.lib.zmi_layernorm_rows(self.x_pre.data_ptr(), self.d, m, self.d, ln[0].data_ptr(),
                                               ln[1].data_ptr(), self.eps, out.data_ptr(), self.d, self.sptr), "ln")

    def _prefill_layers(self, m: int, max_pos: int):
        """The m = 2 x S prefill rows through every layer, with the decode step's kernels (same per-row
        arithmetic; each LayerNorm computed once per layer by zmi_layernorm_rows, identical bits)."""
        d, qd = self.d, self.H * self.hd
        qkv_n = (self.H + 2 * self.Hkv) * self.hd
        xn = self.xn_pre
        for i, lw in enumerate(self.w["layers"]):
            self._ln_pre(m, (lw["ln1_w"], lw["ln1_b"]), xn)
            self._run_gemv(self._gemv(lw["qkv"], xn, m, qkv_n, d, _lib.EPI_QKV, self.q_pre, qd,
                                      kv=(self.kc[i], self.vc[i]), row_kv=self.row_kv_pre, row_pos=self.row_pos_pre))
            self._attention(i, self.q_pre, m, self.row_kv_pre, self.row_pos_pre, max_pos, self.attn_pre)
            self._run_gemv(self._gemv(lw["out"], self.attn_pre, m, d, qd, _lib.EPI_RESIDUAL, self.x_pre, d))
            self._ln_pre(m, (lw["ln2_w"], lw["ln2_b"]), xn)
            self._run_gemv(self._gemv(lw["fc1"], xn, m, 2 * self.F, d, _lib.EPI_SWIGLU, self.h_pre, self.F))
            self._run_gemv(self._gemv(lw["fc2"], self.h_pre, m, d, self.F, _lib.EPI_RESIDUAL, self.x_pre, d))

    # ------------------------------------------------------------------ readback
    def slot_state(self, slot: int) -> dict:
        self.stream.synchronize()
        self.check_errors()
        return {k: int(v[slot].item()) for k, v in self.st.items()}

    def read_codes(self, slot: int) -> torch.Tensor:
        """revert_delay_pattern, >=1024 -> 0, truncate to offset-9 (model.py:309-311) -> [1, 9, T] int64."""
        stt = self.slot_state(slot)
        n_audio = stt["total_len"] - 9
        k = stt["offset"] - 9  # python slice end `[..., :offset - 9]`, negative when stopped early by a callback
        t = min(k, n_audio) if k >= 0 else max(n_audio + k, 0)
        with torch.cuda.stream(self.stream):
            out = torch.zeros(N_CODEBOOKS, t, dtype=torch.int64, device=self.dev)
            if t:
                _lib.check(self.lib.zmi_delay_revert(ctypes.byref(self.slots), slot, out.data_ptr(), t, self.sptr),
                           "revert")
        self.stream.synchronize()
        return out.unsqueeze(0)

    def release(self, slot: int):
        self.pos_hi[slot] = 0
        with torch.cuda.stream(self.stream):
            self.st["active"][slot] = 0
            self.row_pos[2 * slot: 2 * slot + 2] = -1


def make_engine(cfg: ZonosConfig, device="cuda", max_slots: int = 1, max_seqlen: int = 2048,
                max_prefill: int = 512) -> HipEngine:
    """The engine for a config's backbone: HipEngine (transformer) or HybridEngine (Mamba2 + MHA)."""
    if cfg.backbone.ssm_cfg:
        from .hybrid import HybridEngine
        return HybridEngine(cfg, device, max_slots, max_seqlen, max_prefill)
    return HipEngine(cfg, device, max_slots, max_seqlen, max_prefill)
