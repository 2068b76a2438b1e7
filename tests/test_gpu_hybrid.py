"""Hybrid backbone (Zonos-v0.1-hybrid, reference zonos/backbone/_mamba_ssm.py:9-57) on the HIP kernels
vs oracle/hybrid_cpu.py. PARITY UNPINNED: mamba-ssm 2.2.4 is absent, so the oracle restates its
published algorithm; these tests hold the HIP path to that restatement (kernel by kernel, then the
whole model teacher-forced) and to batch invariance. Tolerances are stated per test in bf16 ulps.
"""
import ctypes

import pytest
import torch

from oracle.hybrid_cpu import (OracleHybrid, add_layernorm, gated_rmsnorm, mamba2_scan_ref, mamba2_step_ref)
from tests.helpers import synthetic_weights
from zonos_vibes_amd.config import hybrid_config, tiny_hybrid

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ulp(x):
    return torch.ldexp(torch.ones_like(x), torch.frexp(x.abs().clamp_min(1e-30))[1] - 8)


def _ulps(got, ref):
    """|got - ref| in bf16 ulps of ref (floored at the ulp of 1e-3 of the tensor's scale)."""
    got, ref = got.float().cpu(), ref.float().cpu()
    floor = _ulp(torch.tensor(ref.abs().max().item() * 1e-3))
    return ((got - ref).abs() / torch.maximum(_ulp(ref), floor)).max().item()


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16)


def _lib():
    from zonos_vibes_amd import _lib
    return _lib, _lib.lib()


def test_add_layernorm_matches_oracle():
    L, lib = _lib()
    for k in (512, 2048):
        m = 5
        hid, res = _bf(m, k, seed=1), _bf(m, k, scale=3.0, seed=2)
        w, b = _bf(k, scale=0.1, seed=3) + 1, _bf(k, scale=0.02, seed=4)
        for first in (True, False):
            r = res.to(DEV).clone()
            out = torch.empty(m, k, dtype=torch.bfloat16, device=DEV)
            hd = None if first else hid.to(DEV)
            wd, bd = w.to(DEV), b.to(DEV)
            L.check(lib.zmi_add_layernorm(None if first else hd.data_ptr(), k, r.data_ptr(), k, m, k, wd.data_ptr(),
                                          bd.data_ptr(), 1e-5, out.data_ptr(), k, 1, 0))
            torch.cuda.synchronize()
            ref_y, ref_r = add_layernorm(res if first else hid, None if first else res, w, b, 1e-5)
            assert torch.equal(r.cpu(), ref_r)            # bf16(fp32 sum): exact
            assert _ulps(out, ref_y) <= 2.0


def test_gated_rmsnorm_matches_oracle():
    L, lib = _lib()
    for k in (1024, 4096):
        m = 3
        y, z, w = _bf(m, k, seed=5), _bf(m, k, scale=2.0, seed=6), _bf(k, scale=0.1, seed=7) + 1
        out = torch.empty(m, k, dtype=torch.bfloat16, device=DEV)
        yd, zd, wd = y.to(DEV), z.to(DEV), w.to(DEV)
        L.check(lib.zmi_gated_rmsnorm(yd.data_ptr(), k, zd.data_ptr(), k, m, k, wd.data_ptr(), 1e-5, out.data_ptr(), k,
                                      0))
        torch.cuda.synchronize()
        assert _ulps(out, gated_rmsnorm(y, z, w)) <= 2.0


def _mamba_params(md, seed):
    g = torch.Generator().manual_seed(seed)
    nh, cd = md["nheads"], md["conv_dim"]
    cw = ((torch.rand(cd, md["d_conv"], generator=g) - 0.5)).to(torch.bfloat16)
    cb = (torch.randn(cd, generator=g) * 0.1).to(torch.bfloat16)
    dtb = (torch.rand(nh, generator=g) * 2 - 3).to(torch.bfloat16).float()
    A = -torch.exp((torch.rand(nh, generator=g) * 2.77).to(torch.bfloat16).float())
    D = (1 + 0.1 * torch.randn(nh, generator=g)).to(torch.bfloat16).float()
    return cw, cb, dtb, A, D


def _args(L, md, zx, cw, cb, dtb, A, D, ring, ssm, y, m, row_pos, row_kv=None):
    a = L.Mamba2Args()
    a.zxbcdt, a.ld_zx, a.M = zx.data_ptr(), md["d_in_proj"], m
    a.d_ssm, a.nheads, a.headdim, a.d_state, a.d_conv, a.ngroups = (md["d_ssm"], md["nheads"], 64, 128, 4, 1)
    a.conv_w, a.conv_b, a.dt_bias, a.A, a.D = cw.data_ptr(), cb.data_ptr(), dtb.data_ptr(), A.data_ptr(), D.data_ptr()
    a.conv_ring, a.ssm, a.y, a.ldy = ring.data_ptr(), ssm.data_ptr(), y.data_ptr(), md["d_ssm"]
    a.row_pos = row_pos.data_ptr()
    a.row_kv = None if row_kv is None else row_kv.data_ptr()
    return a


def test_mamba2_step_matches_oracle():
    """causal_conv1d_update + selective_state_update at positions 0, 1, 2, 7, 530 (ring wrap), one inactive row."""
    L, lib = _lib()
    md = tiny_hybrid().backbone.mamba2_dims()
    cw, cb, dtb, A, D = _mamba_params(md, 11)
    pos = [0, 1, 2, 7, 530, -1]
    m = len(pos)
    zx = _bf(m, md["d_in_proj"], seed=12)
    ring = _bf(m, 4, md["conv_dim"], seed=13)
    ssm = _bf(m, md["nheads"], 64, 128, scale=0.5, seed=14)
    dev = {k: v.to(DEV) for k, v in dict(zx=zx, ring=ring, ssm=ssm, cw=cw, cb=cb, dtb=dtb, A=A, D=D).items()}
    y = torch.zeros(m, md["d_ssm"], dtype=torch.bfloat16, device=DEV)
    rp = torch.tensor(pos, dtype=torch.int32, device=DEV)
    a = _args(L, md, dev["zx"], dev["cw"], dev["cb"], dev["dtb"], dev["A"], dev["D"], dev["ring"], dev["ssm"], y, m, rp)
    L.check(lib.zmi_mamba2_step(ctypes.byref(a), 0), "step")
    torch.cuda.synchronize()
    xbc = zx[:, md["d_ssm"]: 2 * md["d_ssm"] + 256]
    for r, p in enumerate(pos):
        if p < 0:
            assert torch.equal(dev["ssm"][r].cpu(), ssm[r]) and not y[r].any()
            continue
        win = torch.stack([ring[r, (p - 3 + k) & 3] if p - 3 + k >= 0 else torch.zeros_like(ring[r, 0])
                           for k in range(3)] + [xbc[r]], dim=-1)[None]
        ry, rs = mamba2_step_ref(zx[r:r + 1], win, ssm[r:r + 1], cw, cb, dtb, A, D, md)
        assert _ulps(y[r], ry[0]) <= 4.0, (p, _ulps(y[r], ry[0]))
        assert _ulps(dev["ssm"][r], rs[0]) <= 1.0
        assert torch.equal(dev["ring"][r, p & 3].cpu(), xbc[r])          # raw input into slot p % 4
        for k in range(1, 4):
            assert torch.equal(dev["ring"][r, (p - k) & 3].cpu(), ring[r, (p - k) & 3])


@pytest.mark.parametrize("form", ["scan", "scan_ws", "scan_ssd"])
@pytest.mark.parametrize("seq_len", [1, 3, 45, 161, 256, 257])
def test_mamba2_scan_matches_oracle(seq_len, form):
    """Mamba2.forward from an empty cache for two sequences (tile edges at 32 positions; 161 = C4's prefill), by the
    single-workgroup scan (zmi_mamba2_scan), the parallel form (zmi_mamba2_scan_ws: conv launch + 4 workgroups per
    (sequence, head), fused multiply-adds) and the quadratic SSD form (scan_ws with ZMI_OPT_SCAN_PQ = 0: MFMA tiles of
    C B^T, the decay matrix and the state sum; sequences past 256 positions fall back to the 4-workgroup scan): y
    within 4 bf16 ulps, the final state within 1."""
    if seq_len > 161 and form == "scan":
        pytest.skip("the single-workgroup scan is covered to 161")
    L, lib = _lib()
    md = tiny_hybrid().backbone.mamba2_dims()
    cw, cb, dtb, A, D = _mamba_params(md, 21)
    zx = _bf(2, seq_len, md["d_in_proj"], seed=22)
    dev = {k: v.to(DEV) for k, v in dict(cw=cw, cb=cb, dtb=dtb, A=A, D=D).items()}
    zxd = zx.reshape(2 * seq_len, -1).to(DEV)
    ring = torch.full((2, 4, md["conv_dim"]), 7.0, dtype=torch.bfloat16, device=DEV)  # stale data must go
    ssm = torch.full((2, md["nheads"], 64, 128), 3.0, dtype=torch.bfloat16, device=DEV)
    y = torch.zeros(2 * seq_len, md["d_ssm"], dtype=torch.bfloat16, device=DEV)
    rp = torch.arange(seq_len, dtype=torch.int32, device=DEV).repeat(2)
    rk = torch.tensor([0] * seq_len + [1] * seq_len, dtype=torch.int32, device=DEV)
    a = _args(L, md, zxd, dev["cw"], dev["cb"], dev["dtb"], dev["A"], dev["D"], ring, ssm, y, 2 * seq_len, rp, rk)
    if form == "scan":
        L.check(lib.zmi_mamba2_scan(ctypes.byref(a), seq_len, 0), "scan")
    else:
        nb = int(lib.zmi_mamba2_scan_ws_bytes(2 * seq_len, md["d_ssm"], md["nheads"]))
        ws = torch.full((nb,), 0xA5, dtype=torch.uint8, device=DEV)  # stale workspace must not matter
        old = lib.zmi_get_option(L.OPT_SCAN_PQ)
        lib.zmi_set_option(L.OPT_SCAN_PQ, 0 if form == "scan_ssd" else 4)  # the library default is the SSD form
        try:
            L.check(lib.zmi_mamba2_scan_ws(ctypes.byref(a), seq_len, ws.data_ptr(), nb, 0), form)
            assert lib.zmi_mamba2_scan_ws(ctypes.byref(a), seq_len, ws.data_ptr(), nb - 1, 0) != 0  # too small: refused
        finally:
            lib.zmi_set_option(L.OPT_SCAN_PQ, old)
    torch.cuda.synchronize()
    ry, rs, rconv = mamba2_scan_ref(zx, cw, cb, dtb, A, D, md)
    assert _ulps(y.view(2, seq_len, -1), ry) <= 4.0
    assert _ulps(ssm, rs) <= 1.0
    for sq in range(2):  # slot q % 4 holds the raw input of q (zero for q < 0): the last d_conv inputs
        for k in range(4):
            q = seq_len - 4 + k
            assert torch.equal(ring[sq, q & 3].cpu(), rconv[sq, :, k])


def _teacher_forced(cfg, n_steps, lc=8, seed=0, max_err_ulps=None):
    """Prefill + n_steps decode steps along the oracle's greedy trajectory; per step the max |HIP - oracle|
    CFG'd logit error in bf16 ulps of the step's max |logit|. Returns (errors, decisions that differ where
    the oracle's top-1 / top-2 margin exceeds twice the error bound)."""
    from zonos_vibes_amd.engine import SamplingParams
    from zonos_vibes_amd.model import Zonos
    w = synthetic_weights(cfg, seed=seed)
    o = OracleHybrid(cfg, w)
    cond = _bf(2, lc, cfg.backbone.d_model, seed=31)
    raw = []
    o.generate(cond, max_new_tokens=n_steps, sampling_params=dict(temperature=0.0, repetition_penalty=1.0),
               raw_trace=raw)
    dl = o.last_delayed[0]
    m = Zonos.synthetic(cfg, DEV, seed=seed, max_seqlen=lc + n_steps + 32, max_prefill=64)
    e = m.engine
    e.prefill(0, cond.to(DEV), None, n_steps, SamplingParams(temperature=0.0, repetition_penalty=1.0))
    e.stream.synchronize()

    def cfg_logits(rows):
        c, u = rows[0].float().cpu(), rows[1].float().cpu()
        lg = u + (c - u) * 2.0
        lg[..., 1025:] = -torch.inf
        return lg

    got = [cfg_logits(e.logits_pre)]
    for _ in range(len(raw) - 1):
        with torch.cuda.stream(e.stream):
            e.delayed[0, :, : dl.shape[-1]] = dl.to(DEV, torch.int32)
            for k, v in (("active", 1), ("stopping", 0), ("remaining", 1000)):
                e.st[k][0] = v
            e.refresh_inputs()
        e.step(1, use_graph=False, slots=1)
        e.stream.synchronize()
        lg = cfg_logits(e.logits[0:2])
        lg[1:, 1024] = -torch.inf  # the reference's EOS bias on codebooks 1..8 (model.py:266-268)
        got.append(lg)
    errs, flips = [], 0
    for g, r in zip(got, raw):
        r = r[0]
        fin = torch.isfinite(r)
        scale = _ulp(r[fin].abs().max())
        err = ((g - r).abs()[fin].max() / scale).item()
        errs.append(err)
        top2 = r[:, :1025].topk(2, dim=-1)
        margin = (top2.values[:, 0] - top2.values[:, 1]) / scale
        det = margin > 2 * (max_err_ulps or err)
        flips += int((g[:, :1025].argmax(-1) != top2.indices[:, 0])[det].sum())
    return errs, flips


def test_tiny_hybrid_teacher_forced_logits_and_decisions():
    """Prefill (scan) + 24 decode steps (step kernel, MHA on the rotated KV cache), 4 layers with the attention
    layer in the middle; logits within 24 bf16 ulps of the step's max |logit| (the GEMV and attention
    reduction orders differ from the CPU's), and every decision with a margin above twice that identical."""
    errs, flips = _teacher_forced(tiny_hybrid(), 24, max_err_ulps=24)
    assert max(errs) <= 24, errs
    assert flips == 0


def test_tiny_hybrid_with_mlp_layers():
    """d_intermediate / attn_mlp_d_intermediate > 0: the Block's second add + LayerNorm and GatedMLP."""
    errs, flips = _teacher_forced(tiny_hybrid(3, (1,), d_intermediate=1024, attn_mlp_d_intermediate=512), 8,
                                  max_err_ulps=24)
    assert max(errs) <= 24, errs
    assert flips == 0


def test_full_width_hybrid_layers_teacher_forced():
    """Zonos-v0.1-hybrid widths (d 2048, d_ssm 4096, 64 Mamba2 heads, MHA 16/4) at 3 layers."""
    errs, flips = _teacher_forced(hybrid_config(2048, 3, [1], 16, 4), 6, lc=12, max_err_ulps=32)
    assert max(errs) <= 32, errs
    assert flips == 0


def test_hybrid_generate_batch_equals_single():
    """Batch invariance of every hybrid kernel: three utterances through 3 slots == generate() each."""
    from zonos_vibes_amd.model import Zonos
    cfg = tiny_hybrid()
    m = Zonos.synthetic(cfg, DEV, seed=3, max_slots=3, max_seqlen=96, max_prefill=32)
    conds = [_bf(2, lc, cfg.backbone.d_model, seed=40 + lc).to(DEV) for lc in (5, 9, 7)]
    n = [20, 14, 30]
    sp = dict(temperature=0.0)
    batch = m.generate_batch(conds, max_new_tokens=n, sampling_params=sp, seeds=[1, 2, 3], max_slots=3)
    for c, k, b in zip(conds, n, batch):
        single = m.generate(c, max_new_tokens=k, sampling_params=sp, progress_bar=False)
        assert torch.equal(single.cpu(), b.cpu())


def test_hybrid_full_dims_generate_and_backbone_plugin():
    """Zonos-v0.1-hybrid dims (46 layers, 2.3 GB bf16): generate() through the hipGraph decode loop, and the
    BACKBONES['hip'] plugin's forward over the 40 conditioning rows of both CFG halves equals, bit for bit, the
    norm_f'd hidden states of the engine's own prefill of the same rows (the prefill carries one more row, the
    embedded first frame, which causal attention and the Mamba2 scan keep out of the earlier rows)."""
    from zonos_vibes_amd.backbone import BACKBONES
    from zonos_vibes_amd.config import InferenceParams, zonos_v01_hybrid
    from zonos_vibes_amd.engine import SamplingParams
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_hybrid()
    m = Zonos.synthetic(cfg, DEV, seed=0, zero_eos=True, max_seqlen=256, max_prefill=64)
    lc = 40
    cond = _bf(2, lc, 2048, seed=50).to(DEV)
    codes = m.generate(cond, max_new_tokens=64, sampling_params=dict(temperature=0.0), progress_bar=False)
    assert codes.shape == (1, 9, 64) and int(codes.max()) < 1024
    bb = BACKBONES["hip"](cfg.backbone)
    bb.load_state_dict({k[len("backbone."):]: v for k, v in synthetic_weights_gpu(m).items()})
    cache = bb.allocate_inference_cache(2, 64)
    assert len(cache) == 46
    out = bb(cond, InferenceParams(64, 2, key_value_memory_dict=cache))
    assert out.shape == (2, lc, 2048) and torch.isfinite(out.float()).all()
    e = m.engine
    s_len = e.prefill(0, cond, None, 8, SamplingParams(temperature=0.0))
    assert s_len == lc + 1
    ref = torch.empty(2 * s_len, 2048, dtype=torch.bfloat16, device=DEV)
    with torch.cuda.stream(e.stream):
        e.final_norm_pre(2 * s_len, ref)
    e.stream.synchronize()
    e.release(0)
    assert torch.equal(out[0], ref[:lc])
    assert torch.equal(out[1], ref[s_len: s_len + lc])


def synthetic_weights_gpu(m):
    """The model's synthetic backbone weights regenerated on the GPU (same stream as init_synthetic)."""
    from zonos_vibes_amd import _lib as L
    from zonos_vibes_amd import synthetic as syn
    lib = L.lib()
    out = {}
    for sp in syn.zonos_specs(m.config):
        if not sp.name.startswith("backbone."):
            continue
        t = torch.empty(sp.shape, dtype=torch.bfloat16, device=DEV)
        L.check(lib.zmi_fill_uniform(t.data_ptr(), sp.numel, syn.tensor_key(0, sp.name), sp.scale, sp.offset, 0, 0))
        out[sp.name] = t
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("rows", [1, 2, 4, 5, 8])
def test_norm_prologues_equal_standalone_kernels(rows):
    """The decode plan's fused prologues give the prefill path's bits: GEMV(ADDLN) == zmi_add_layernorm +
    plain GEMV (and its residual output); GEMV(GRMS) on the step kernel's y and f32 gate == zmi_gated_rmsnorm
    (y, z) + plain GEMV (up to 4 rows)."""
    from tests.test_gpu_kernels import pack, stream_ptr
    from zonos_vibes_amd.config import zonos_v01_hybrid
    L, lib = _lib()
    for kind, K, N in (("addln", 2048, 8512), ("addln", 512, 2320), ("grms", 4096, 2048), ("grms", 1024, 512)):
        if kind == "grms" and rows > 4:
            continue
        Wp, n_pad = pack(_bf(N, K, scale=0.03, seed=90 + K).to(DEV))
        w, b = (_bf(K, scale=0.1, seed=93) + 1).to(DEV), _bf(K, scale=0.02, seed=94).to(DEV)
        fused = torch.zeros(rows, n_pad, dtype=torch.bfloat16, device=DEV)
        plain = torch.zeros_like(fused)
        nrm = torch.zeros(rows, K, dtype=torch.bfloat16, device=DEV)

        def gemv(X, pro, out, aux=None, ld_aux=0, res_out=None):
            a = L.GemvArgs()
            a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), X.data_ptr(), rows, n_pad, K, K
            a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), n_pad, n_pad, 1e-5
            if pro:
                a.pro, a.aux, a.ld_aux, a.res_out = pro, aux.data_ptr(), ld_aux, L.ptr(res_out)
                a.ln_w = w.data_ptr()
                a.ln_b = b.data_ptr() if pro == L.PRO_ADDLN else None
            L.check(lib.zmi_gemv_launch(ctypes.byref(a), L.EPI_STORE, stream_ptr()), kind)

        if kind == "addln":
            x = _bf(rows, K, scale=1.5, seed=91).to(DEV)
            aux = _bf(rows, K, scale=2.0, seed=92).to(DEV)
            r_out = torch.zeros_like(aux)
            gemv(x, L.PRO_ADDLN, fused, aux, K, r_out)
            r_ref = aux.clone()
            L.check(lib.zmi_add_layernorm(x.data_ptr(), K, r_ref.data_ptr(), K, rows, K, w.data_ptr(), b.data_ptr(),
                                          1e-5, nrm.data_ptr(), K, 1, stream_ptr()))
        else:  # y and the gate from the Mamba2 step kernel itself
            md = (zonos_v01_hybrid() if K == 4096 else tiny_hybrid()).backbone.mamba2_dims()
            cw, cb, dtb, A, D = (t.to(DEV) for t in _mamba_params(md, 95))
            zx = _bf(rows, md["d_in_proj"], scale=2.0, seed=96).to(DEV)
            ring = torch.zeros(rows, 4, md["conv_dim"], dtype=torch.bfloat16, device=DEV)
            ssm = _bf(rows, md["nheads"], 64, 128, scale=0.5, seed=97).to(DEV)
            y = torch.zeros(rows, K, dtype=torch.bfloat16, device=DEV)
            gz = torch.zeros(rows, K, dtype=torch.float32, device=DEV)
            rp = torch.full((rows,), 9, dtype=torch.int32, device=DEV)
            a = _args(L, md, zx, cw, cb, dtb, A, D, ring, ssm, y, rows, rp)
            a.gz = gz.data_ptr()
            L.check(lib.zmi_mamba2_step(ctypes.byref(a), stream_ptr()), "step")
            gemv(y, L.PRO_GRMS, fused, gz, K)
            L.check(lib.zmi_gated_rmsnorm(y.data_ptr(), K, zx.data_ptr(), md["d_in_proj"], rows, K, w.data_ptr(), 1e-5,
                                          nrm.data_ptr(), K, stream_ptr()))
        gemv(nrm, 0, plain)
        torch.cuda.synchronize()
        assert torch.equal(fused, plain), (kind, K)
        if kind == "addln":
            assert torch.equal(r_out, r_ref), (kind, K)


def test_mamba_block_launch_bit_identical_to_separate():
    """zmi_mamba_block (in_proj + Mamba2 step in one launch, granule hand-off) decodes exactly as the separate
    in_proj GEMV + zmi_mamba2_step: one utterance (2 rows, fused gate) and 8 slots (16 rows) at full width."""
    from zonos_vibes_amd.model import Zonos
    cfg = hybrid_config(2048, 3, [1], 16, 4)
    m = Zonos.synthetic(cfg, DEV, seed=4, max_slots=8, max_seqlen=96, max_prefill=32)
    conds = [_bf(2, lc, 2048, seed=60 + lc).to(DEV) for lc in (5, 9, 7, 12, 6, 8, 11, 10)]
    sp = dict(temperature=0.0)
    res = []
    for fused in (True, False):
        m.engine.mamba_block = fused
        m.engine._build_plan()
        one = m.generate(conds[0], max_new_tokens=30, sampling_params=sp, progress_bar=False)
        many = m.generate_batch(conds, max_new_tokens=[20, 14, 30, 9, 25, 17, 12, 22], sampling_params=sp,
                                seeds=list(range(8)), max_slots=8)
        m.engine.check_errors()
        res.append((one.cpu(), [c.cpu() for c in many]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


def test_attn_block_addln_bit_identical_to_separate():
    """The MHA blocks' QKV (ADDLN prologue) + attention as one zmi_attn_block launch decode exactly as the
    separate QKV GEMV + attention kernel: one utterance (2 rows) and 8 slots (16 rows) at full width."""
    from zonos_vibes_amd.model import Zonos
    cfg = hybrid_config(2048, 3, [1], 16, 4)
    m = Zonos.synthetic(cfg, DEV, seed=5, max_slots=8, max_seqlen=96, max_prefill=32)
    conds = [_bf(2, lc, 2048, seed=80 + lc).to(DEV) for lc in (5, 9, 7, 12, 6, 8, 11, 10)]
    sp = dict(temperature=0.0)
    res = []
    for fused in (True, False):
        m.engine.attn_block = fused
        m.engine.attn_block_rows = 16  # the fused forms at 16 rows too (the default stops at 8: speed only)
        m.engine._build_plan()
        assert any(it[0] == "attnblk" for it in m.engine._plan(2, m.engine._segments(1, 1)[0][1])) == fused
        one = m.generate(conds[0], max_new_tokens=30, sampling_params=sp, progress_bar=False)
        many = m.generate_batch(conds, max_new_tokens=[20, 14, 30, 9, 25, 17, 12, 22], sampling_params=sp,
                                seeds=list(range(8)), max_slots=8)
        m.engine.check_errors()
        res.append((one.cpu(), [c.cpu() for c in many]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)
