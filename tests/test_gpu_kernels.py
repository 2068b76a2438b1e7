"""Kernel-level parity of the HIP C ABI against the oracle / fp32 references (MI355X only)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from oracle import zonos_cpu as oz
from tests.helpers import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    from zonos_vibes_amd import _lib as L
    return L


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


def pack(W, mode=0, n_pad=None):
    L = _lib()
    n, k = W.shape
    n_pad = n_pad or (n + 7) // 8 * 8
    out = torch.empty(n_pad * k, dtype=torch.bfloat16, device=DEV)
    L.check(L.lib().zmi_pack_weight(W.data_ptr(), out.data_ptr(), n, k, n_pad, mode, stream_ptr()))
    return out, n_pad


def gemv(W, X, epi, out, ldo, n_valid=None, ln=None, mode=0, extra=None, groups=0, packed=None):
    L = _lib()
    Wp, n_pad = packed if packed is not None else pack(W, mode)
    M, K = X.shape
    a = L.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), X.data_ptr(), M, n_pad, K, K
    a.groups = groups
    if ln is not None:
        a.ln_w, a.ln_b, a.eps = ln[0].data_ptr(), ln[1].data_ptr(), 1e-5
    a.out, a.ldo = out.data_ptr(), ldo
    a.n_valid = W.shape[0] if n_valid is None else n_valid
    if extra:
        extra(a)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(a), epi, stream_ptr()), "gemv")
    torch.cuda.synchronize()
    return out


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1).mul(scale).to(torch.bfloat16).to(DEV)


@pytest.mark.parametrize("M,N,K", [(1, 64, 512), (2, 3072, 2048), (5, 2048, 8192), (8, 9248, 2048), (16, 256, 512),
                                   (33, 512, 1024), (130, 256, 2048), (2, 2048, 8192), (1, 512, 4096), (19, 136, 8192)])
def test_gemv_f32_sums_match_fp64(M, N, K):
    L = _lib()
    W, X = rnd(N, K, scale=0.05, seed=1), rnd(M, K, seed=2)
    out = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    gemv(W, X, L.EPI_F32, out, N)
    ref = X.double() @ W.double().t()
    bound = (X.double().abs() @ W.double().abs().t()) * 2e-6 + 1e-30
    assert ((out.double() - ref).abs() <= bound).all()


@pytest.mark.parametrize("K,ln", [(2048, True), (2048, False), (8192, False), (512, True)])
def test_gemv_is_batch_invariant(K, ln):
    """A row's result is bit-identical whatever batch it is computed in (any M, any row tile,
    any position inside the tile): SURVEY.md §0.3, the reference's batch_size=1 semantics."""
    L = _lib()
    N = 1024
    W = rnd(N, K, scale=0.05, seed=3)
    big = 130
    X = rnd(big, K, scale=2.0, seed=4)
    lnp = (rnd(K, scale=0.1, seed=10) + 1, rnd(K, scale=0.02, seed=11)) if ln else None
    packed = pack(W)
    ref = torch.zeros(big, N, dtype=torch.float32, device=DEV)
    gemv(W, X, L.EPI_F32, ref, N, ln=lnp, packed=packed)
    for lo, hi in [(0, 1), (0, 2), (5, 12), (0, 16), (3, 20), (17, 50), (64, 130), (129, 130)]:
        small = torch.zeros(hi - lo, N, dtype=torch.float32, device=DEV)
        gemv(W, X[lo:hi].contiguous(), L.EPI_F32, small, N, ln=lnp, packed=packed)
        assert torch.equal(small, ref[lo:hi]), (lo, hi)
    # the column-group choice (2 groups per block are built for the LayerNorm'd K = 2048 shape)
    # does not change a column's arithmetic either
    for g in ((1, 2) if (K, ln) == (2048, True) else (1,)):
        alt = torch.zeros(big, N, dtype=torch.float32, device=DEV)
        gemv(W, X, L.EPI_F32, alt, N, ln=lnp, packed=packed, groups=g)
        assert torch.equal(alt, ref)


PROD_SHAPES = {  # Zonos-v0.1 decode GEMVs: (N, K, LayerNorm'd, epilogue, pack mode)
    "qkv": (3072, 2048, True, "qkv", 0), "out_proj": (2048, 2048, False, "f32", 0),
    "fc1": (16384, 2048, True, "swiglu", 1), "fc2": (2048, 8192, False, "f32", 0),
    "heads": (9248, 2048, True, "f32", 0), "out_proj_residual": (2048, 2048, False, "residual", 0),
    "fc2_residual": (2048, 8192, False, "residual", 0)}


@pytest.mark.parametrize("rows_opt", [1, 3])
@pytest.mark.parametrize("name", list(PROD_SHAPES))
def test_gemv_batch_invariant_production_shapes(name, rows_opt):
    """The many-row GEMV geometries (the K = 2048 many-row form with its tiles DMA'd two ahead, or the
    4-column-group tile loop, by row count and width; per-shape workgroup targets) give every row the bits
    of the decode-step launch (1-16 rows, single tile, LayerNorm prologue) at the production shapes,
    epilogues included; the many-row plan LayerNorms its rows once per layer (zmi_layernorm_rows), the
    decode plan in the GEMV prologue: generate_batch == generate rests on exactly this. The row ranges
    cross the many-row form's selection bounds (32, 64 rows). rows_opt 3: the many-row form's dense-pair MFMAs
    (ZMI_OPT_GEMM_ROWS bit 1)."""
    L = _lib()
    old = L.lib().zmi_get_option(L.OPT_GEMM_ROWS)
    L.lib().zmi_set_option(L.OPT_GEMM_ROWS, rows_opt)
    try:
        _batch_invariant_production_shape(L, name)
    finally:
        L.lib().zmi_set_option(L.OPT_GEMM_ROWS, old)


def _batch_invariant_production_shape(L, name):
    from zonos_vibes_amd.engine import rope_table
    N, K, ln, epi, mode = PROD_SHAPES[name]
    big = 128
    W = rnd(N, K, scale=0.03, seed=30)
    X = rnd(big, K, scale=2.0, seed=31)
    lnp = ((rnd(K, scale=0.1, seed=32) + 1).contiguous(), rnd(K, scale=0.02, seed=33)) if ln else None
    packed = pack(W, mode)
    rope = rope_table(128).to(DEV)
    smax = 160
    pos_all = torch.randint(0, smax, (big,), generator=torch.Generator().manual_seed(34), dtype=torch.int32).to(DEV)
    res_all = rnd(big, N, scale=4.0, seed=35)

    def run(lo, hi, pre_ln):
        m = hi - lo
        xs = X[lo:hi].contiguous()
        if pre_ln:  # the many-row plan: LayerNorm once, then the plain GEMV
            xn = torch.zeros(m, K, dtype=torch.bfloat16, device=DEV)
            L.check(L.lib().zmi_layernorm_rows(xs.data_ptr(), K, m, K, lnp[0].data_ptr(), lnp[1].data_ptr(), 1e-5,
                                               xn.data_ptr(), K, stream_ptr()))
            xs, use_ln = xn, None
        else:
            use_ln = lnp
        if epi == "f32":
            out = torch.zeros(m, N, dtype=torch.float32, device=DEV)
            gemv(W, xs, L.EPI_F32, out, N, ln=use_ln, packed=packed)
            return (out,)
        if epi == "swiglu":
            out = torch.zeros(m, N // 2, dtype=torch.bfloat16, device=DEV)
            gemv(W, xs, L.EPI_SWIGLU, out, N // 2, ln=use_ln, packed=packed)
            return (out,)
        if epi == "residual":  # out holds the residual stream x on entry, x + bf16(linear(h)) on exit
            out = res_all[lo:hi].clone()
            gemv(W, xs, L.EPI_RESIDUAL, out, N, ln=use_ln, packed=packed)
            return (out,)
        q = torch.zeros(m, 2048, dtype=torch.bfloat16, device=DEV)
        kc = torch.zeros(m, 4, smax, 128, dtype=torch.bfloat16, device=DEV)
        vt = torch.zeros(m, 4, 128, smax, dtype=torch.bfloat16, device=DEV)
        row_kv = torch.arange(m, dtype=torch.int32, device=DEV)
        row_pos = pos_all[lo:hi].contiguous()

        def extra(a):
            a.row_kv, a.row_pos, a.k_cache, a.v_cache = row_kv.data_ptr(), row_pos.data_ptr(), kc.data_ptr(), vt.data_ptr()
            a.smax, a.hq, a.hkv, a.hd, a.rope = smax, 16, 4, 128, rope.data_ptr()
        gemv(W, xs, L.EPI_QKV, q, 2048, ln=use_ln, packed=packed, extra=extra)
        return q, kc, vt

    ref = run(0, big, ln)
    for lo, hi in [(0, 2), (0, 16), (6, 8), (5, 21), (100, 116), (126, 128), (16, 128), (0, 64), (3, 36), (60, 125),
                   (1, 66)]:
        got = run(lo, hi, ln and hi - lo > 4)
        for r, g in zip(ref, got):
            assert torch.equal(g, r[lo:hi]), (name, lo, hi)


@pytest.mark.parametrize("K,M", [(2048, 2), (2048, 16), (2048, 37), (512, 5), (1024, 3)])
def test_layernorm_rows_equals_gemv_prologue(K, M):
    """zmi_layernorm_rows (norm_f of the backbone plugin) and the GEMV LayerNorm prologue share one
    arithmetic (zmi_common.h): a plain GEMV of the normalised rows equals the LayerNorm'd GEMV."""
    L = _lib()
    N = 256
    W, X = rnd(N, K, scale=0.05, seed=14), rnd(M, K, scale=3.0, seed=15)
    lw, lb = (rnd(K, scale=0.2, seed=16) + 1).contiguous(), rnd(K, scale=0.05, seed=17)
    xn = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
    L.check(L.lib().zmi_layernorm_rows(X.data_ptr(), K, M, K, lw.data_ptr(), lb.data_ptr(), 1e-5, xn.data_ptr(), K,
                                       stream_ptr()))
    packed = pack(W)
    a = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    b = torch.zeros(M, N, dtype=torch.float32, device=DEV)
    gemv(W, X, L.EPI_F32, a, N, ln=(lw, lb), packed=packed)
    gemv(W, xn, L.EPI_F32, b, N, packed=packed)
    assert torch.equal(a, b)
    ref = F.layer_norm(X.float().cpu(), (K,), lw.float().cpu(), lb.float().cpu(), 1e-5)
    assert _ulp_close(xn, ref, 1) > 0.99


def _ulp_close(a, b, ulps=1):
    a, b = a.float().cpu(), b.float().cpu()
    ulp = torch.ldexp(torch.ones_like(b), torch.frexp(b.abs().clamp_min(1e-30))[1] - 8)
    return ((a - b).abs() <= ulps * ulp + 1e-30).float().mean().item()


def test_gemv_store_and_residual_match_linear():
    L = _lib()
    W, X = rnd(512, 1024, scale=0.05, seed=5), rnd(6, 1024, seed=6)
    out = torch.zeros(6, 512, dtype=torch.bfloat16, device=DEV)
    gemv(W, X, L.EPI_STORE, out, 512)
    ref = F.linear(X.cpu(), W.cpu())
    assert _ulp_close(out, ref) > 0.999
    res = rnd(6, 512, seed=7)
    res_ref = res.cpu() + ref
    gemv(W, X, L.EPI_RESIDUAL, res, 512)
    assert _ulp_close(res, res_ref) > 0.999


def test_gemv_layernorm_prologue_and_swiglu():
    L = _lib()
    K, Fh = 512, 1024
    W = rnd(2 * Fh, K, scale=0.05, seed=8)
    X = rnd(3, K, scale=2.0, seed=9)
    lw, lb = rnd(K, scale=0.1, seed=10) + 1, rnd(K, scale=0.02, seed=11)
    out = torch.zeros(3, Fh, dtype=torch.bfloat16, device=DEV)
    gemv(W, X, L.EPI_SWIGLU, out, Fh, ln=(lw.contiguous(), lb), mode=L.PACK_SWIGLU)
    xn = F.layer_norm(X.cpu(), (K,), lw.cpu(), lb.cpu(), 1e-5)
    y, g = F.linear(xn, W.cpu()).chunk(2, dim=-1)
    ref = y * F.silu(g)
    err = (out.float().cpu() - ref.float()).abs()
    assert err.max() < 0.02 * ref.float().abs().max()
    assert _ulp_close(out, ref, ulps=2) > 0.97


def test_gemv_qkv_rope_kv_write():
    L = _lib()
    from zonos_vibes_amd.engine import rope_table
    d, H, Hkv, hd, smax = 512, 4, 1, 128, 64
    n = (H + 2 * Hkv) * hd
    W, X = rnd(n, d, scale=0.05, seed=12), rnd(2, d, seed=13)
    rope = rope_table(hd).to(DEV)
    kc = torch.zeros(2, Hkv, smax, hd, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(2, Hkv, hd, smax, dtype=torch.bfloat16, device=DEV)
    q = torch.zeros(2, H * hd, dtype=torch.bfloat16, device=DEV)
    row_kv = torch.tensor([0, 1], dtype=torch.int32, device=DEV)
    row_pos = torch.tensor([5, 37], dtype=torch.int32, device=DEV)

    def extra(a):
        a.row_kv, a.row_pos, a.k_cache, a.v_cache = row_kv.data_ptr(), row_pos.data_ptr(), kc.data_ptr(), vc.data_ptr()
        a.smax, a.hq, a.hkv, a.hd, a.rope = smax, H, Hkv, hd, rope.data_ptr()

    gemv(W, X, L.EPI_QKV, q, H * hd, extra=extra)
    qkv = F.linear(X.cpu(), W.cpu())
    fc = oz.rope_table(16384, hd)
    for r, p in enumerate((5, 37)):
        qq, kk, vv = qkv[r].split([H * hd, hd, hd])
        qr = oz.apply_rope(qq.view(1, 1, H, hd), fc[p:p + 1].unsqueeze(0)).view(-1)
        kr = oz.apply_rope(kk.view(1, 1, 1, hd), fc[p:p + 1].unsqueeze(0)).view(-1)
        assert _ulp_close(q[r], qr, 2) > 0.995
        assert _ulp_close(kc[r, 0, p], kr, 2) > 0.995
        assert _ulp_close(vc[r, 0, :, p], vv, 1) > 0.995  # V cache is stored transposed [hd][position]
        assert kc[r, 0, :p].abs().sum() == 0 and vc[r, 0, :, :p].abs().sum() == 0


def _attention(q, kc, vc, positions, kv_rows=None, hq=16, hkv=4, variant=0):
    """Run zmi_attention_variant (0 = library choice); kc [R][hkv][smax][hd], vc the same cache in the
    kernel's transposed layout."""
    L = _lib()
    hd, smax = kc.shape[-1], kc.shape[-2]
    n = len(positions)
    vt = vc.transpose(-1, -2).contiguous()
    out = torch.zeros(n, hq * hd, dtype=torch.bfloat16, device=DEV)
    rp = torch.tensor(positions, dtype=torch.int32, device=DEV)
    rk = None if kv_rows is None else torch.tensor(kv_rows, dtype=torch.int32, device=DEV)
    work = torch.zeros(L.lib().zmi_attention_work_bytes(n, hq, hkv, hd, smax - 1), dtype=torch.uint8, device=DEV)
    nf = L.lib().zmi_attention_partial_floats(n, hq, hkv, hd, smax - 1)
    po = torch.zeros(nf, dtype=torch.float32, device=DEV)
    plm = torch.zeros(nf // hd * 2, dtype=torch.float32, device=DEV)
    for _ in range(2):  # the second launch checks that the hand-off state re-armed itself
        L.check(L.lib().zmi_attention_variant(q.data_ptr(), hq * hd, kc.data_ptr(), vt.data_ptr(), _lib().ptr(rk),
                                              rp.data_ptr(), n, hq, hkv, hd, smax, smax - 1, out.data_ptr(), hq * hd,
                                              po.data_ptr(), plm.data_ptr(), work.data_ptr(), variant, stream_ptr()))
        torch.cuda.synchronize()
        assert int(work[:4].view(torch.int32).item()) == 0, "cross-chunk hand-off timed out"
    return out


def _check_attention(out, q, kc, vc, positions, kv_rows=None, hq=16, hkv=4):
    from oracle.attention_cpu import attend
    hd = kc.shape[-1]
    for r, p in enumerate(positions):
        kr = r if kv_rows is None else kv_rows[r]
        qq = q[r].view(hq, hd).cpu()
        got = out[r].view(hq, hd).float().cpu()
        ref = attend(qq, kc[kr].cpu(), vc[kr].cpu(), p).float()
        # same blocking and rounding points: equal up to the fp32 accumulation order, which can
        # flip a probability's bf16 rounding (then ~1 bf16 ulp of the output)
        ulp = torch.ldexp(torch.ones_like(ref), torch.frexp(ref.abs().clamp_min(1e-6))[1] - 8)
        err = (got - ref).abs()
        assert (err <= 2 * ulp + 1e-4).float().mean() > 0.995, (p, err.max().item())
        assert err.max() < 2e-2, (p, err.max().item())
        # and against plain fp32 SDPA, the math the op stands for
        sd = F.scaled_dot_product_attention(qq.float().view(1, hq, 1, hd), kc[kr, :, : p + 1].float().cpu().unsqueeze(0),
                                            vc[kr, :, : p + 1].float().cpu().unsqueeze(0), enable_gqa=True).view(hq, hd)
        assert (got - sd).abs().max() < 2e-2, p


@pytest.mark.parametrize("positions", [(0, 1), (63, 64), (65, 200), (511, 7), (512, 513), (1023, 1500)])
def test_attention_matches_reference_blocking(positions):
    H, Hkv, hd, smax = 16, 4, 128, 2048
    R = len(positions)
    kc = rnd(R, Hkv, smax, hd, seed=20)
    vc = rnd(R, Hkv, smax, hd, seed=21)
    q = rnd(R, H * hd, scale=2.0, seed=22)
    out = _attention(q, kc, vc, positions)
    _check_attention(out, q, kc, vc, positions)


@pytest.mark.parametrize("hq,hkv", [(16, 4), (4, 1), (8, 4)])
def test_attention_whole_query_variant_bit_identical_to_chunked(hq, hkv):
    """The whole-query kernel (one workgroup per (query, kv head, dim slice), no cross-workgroup
    exchange) restates the chunked kernel's arithmetic operation for operation: identical bits at
    every position it covers, including chunk / block edges and the last covered position."""
    hd = 128
    lim = _lib().lib().zmi_attention_max_keys_whole()
    smax = lim + 8
    positions = [0, 1, 31, 32, 127, 128, 129, 300, 511, 512, 591, 640, 1023, 1024, 1030, lim - 2, lim - 1]
    R = len(positions)
    kc = rnd(R, hkv, smax, hd, seed=60)
    vc = rnd(R, hkv, smax, hd, seed=61)
    q = rnd(R, hq * hd, scale=3.0, seed=62)
    ref = _attention(q, kc, vc, positions, hq=hq, hkv=hkv, variant=1)
    # the whole-query kernel covers max_pos < lim: give it a cache view whose capacity is lim
    for ds in (4, 8):
        got = _attention(q, kc[:, :, :lim].contiguous(), vc[:, :, :lim].contiguous(), positions, hq=hq, hkv=hkv,
                         variant=ds)
        assert torch.equal(got, ref), (ds, (got != ref).nonzero()[:4].tolist())
    _check_attention(got[[0, 6, 10, 14, R - 1]], q[[0, 6, 10, 14, R - 1]], kc[[0, 6, 10, 14, R - 1]],
                     vc[[0, 6, 10, 14, R - 1]], [positions[i] for i in (0, 6, 10, 14, R - 1)], hq=hq, hkv=hkv)


@pytest.mark.parametrize("variant", [2, 3, 5])
@pytest.mark.parametrize("hq,hkv", [(16, 4), (4, 1), (8, 4)])
def test_attention_split_launch_variants_bit_identical_to_one_launch(hq, hkv, variant):
    """Variant 2 (scores + maxima launch, then the finish launch, no waiting inside either), variant 3 (the
    same, the merge as a third launch) and variant 5 (one workgroup per 512-key block) against variant 1 (one
    launch, one workgroup per 128-key chunk, maxima exchanged by granules): identical bits at chunk / block
    edges and at C5 lengths, with a KV-row table, launched twice (the state a launch leaves must not leak into
    the next)."""
    hd, smax = 128, 5784
    positions = [0, 1, 127, 128, 511, 512, 513, 1023, 1279, 1280, 2047, 2049, 3200, 4100, 5775]
    R = len(positions)
    kc = rnd(R, hkv, smax, hd, seed=63)
    vc = rnd(R, hkv, smax, hd, seed=64)
    q = rnd(R + 2, hq * hd, scale=3.0, seed=65)
    rows = list(range(R)) + [3, R - 1]
    pos = positions + [5000, 17]
    ref = _attention(q, kc, vc, pos, kv_rows=rows, hq=hq, hkv=hkv, variant=1)
    got = _attention(q, kc, vc, pos, kv_rows=rows, hq=hq, hkv=hkv, variant=variant)
    assert torch.equal(got, ref), (got != ref).nonzero()[:4].tolist()
    pick = [0, 6, 12, R - 1, R]
    _check_attention(got[pick], q[pick], kc, vc, [pos[i] for i in pick], kv_rows=[rows[i] for i in pick], hq=hq,
                     hkv=hkv)


def test_attention_long_context_c5_positions():
    """C5 voice-clone lengths: P = 430 prefix frames + 5168 new ones reach ~5.8k positions, 12
    blocks of 512 keys chained through the cross-block maxima and merged in block order."""
    H, Hkv, hd, smax = 16, 4, 128, 5784
    positions = (2047, 2049, 4100, 5775)
    R = len(positions)
    kc = rnd(R, Hkv, smax, hd, seed=30)
    vc = rnd(R, Hkv, smax, hd, seed=31)
    q = rnd(R, H * hd, scale=3.0, seed=32)
    out = _attention(q, kc, vc, positions)
    _check_attention(out, q, kc, vc, positions)


def test_attention_prefill_rows_with_kv_table():
    """Prefill layout: 2 x S query rows, each its own position, reading the KV row of its CFG half."""
    H, Hkv, hd, smax = 4, 1, 128, 640
    S = 600
    kc = rnd(2, Hkv, smax, hd, seed=40)
    vc = rnd(2, Hkv, smax, hd, seed=41)
    pos = [p for p in range(S)] * 2
    rows = [0] * S + [1] * S
    q = rnd(2 * S, H * hd, seed=42)
    out = _attention(q, kc, vc, pos, kv_rows=rows, hq=H, hkv=Hkv)
    pick = [0, 1, 300, 511, 512, 599, S, S + 513, 2 * S - 1]
    _check_attention(out[pick], q[pick], kc, vc, [pos[i] for i in pick], kv_rows=[rows[i] for i in pick], hq=H,
                     hkv=Hkv)


def test_attention_is_batch_invariant():
    H, Hkv, hd, smax = 16, 4, 128, 1200
    positions = [5, 700, 1100, 64, 513, 1000, 999, 2]
    R = len(positions)
    kc = rnd(R, Hkv, smax, hd, seed=50)
    vc = rnd(R, Hkv, smax, hd, seed=51)
    q = rnd(R, H * hd, seed=52)
    full = _attention(q, kc, vc, positions)
    for r in (0, 1, 5):
        one = _attention(q[r:r + 1].contiguous(), kc[r:r + 1].contiguous(), vc[r:r + 1].contiguous(), positions[r:r + 1])
        assert torch.equal(one[0], full[r])


def _slots(S=4, tcap=128):
    L = _lib()
    st = {k: torch.zeros(S, dtype=torch.int32, device=DEV) for k in
          ("active", "pos", "offset", "remaining", "stopping", "step", "total_len")}
    delayed = torch.full((S, 9, tcap), 1025, dtype=torch.int32, device=DEV)
    params = torch.zeros(S * ctypes.sizeof(L.Sampling), dtype=torch.uint8, device=DEV)
    sl = L.Slots(*(st[k].data_ptr() for k in ("active", "pos", "offset", "remaining", "stopping", "step")),
                 delayed.data_ptr(), params.data_ptr(), st["total_len"].data_ptr(), tcap, S)
    return sl, st, delayed, params


def _set_params(params, s, p):
    L = _lib()
    sz = ctypes.sizeof(L.Sampling)
    params[s * sz:(s + 1) * sz].copy_(torch.tensor(bytearray(p), dtype=torch.uint8))


def _run_sampler_on_final_logits(logits, generated, sp, noise=None):
    """Drive the sampler with already-guided logits: cond row = logits, uncond row = 0, cfg 1."""
    L = _lib()
    from zonos_vibes_amd.engine import SamplingParams
    B = logits.shape[0]
    sl, st, delayed, params = _slots(B)
    rows = torch.zeros(2 * B, 9, 1026, device=DEV)
    rows[0::2] = logits.to(DEV)
    g = generated.shape[-1]
    delayed[:, :, :g] = generated.to(DEV, torch.int32)
    st["active"][:] = 1
    st["offset"][:] = g - 1
    st["remaining"][:] = 100
    st["total_len"][:] = 64
    for s in range(B):
        _set_params(params, s, SamplingParams.from_dict(sp, 1.0, 1234 + s).to_c())
    nxt = torch.zeros(B, 9, dtype=torch.int32, device=DEV)
    cnt = torch.zeros(B, dtype=torch.int32, device=DEV)
    nz = None if noise is None else noise.to(DEV).contiguous()
    L.check(L.lib().zmi_sample_step(ctypes.byref(sl), rows.data_ptr(), None if nz is None else nz.data_ptr(),
                                    nxt.data_ptr(), cnt.data_ptr(), 0, 0, B, None, 0, None, None, None,
                                    stream_ptr()))
    torch.cuda.synchronize()
    return nxt.cpu().long().unsqueeze(-1), st, delayed


def test_sampler_greedy_with_penalty_matches_reference():
    t, _ = load_golden("penalty_greedy")
    out, _, _ = _run_sampler_on_final_logits(t["logits"], t["generated"], dict(temperature=0.0))
    assert torch.equal(out, t["greedy"])


def test_sampler_penalty_windows_match_reference():
    """Windows beyond the default 2, the whole history (0) and negative windows: the kernel
    counts every token of generated[..., -window:] (reference sampling.py:99-114)."""
    t, meta = load_golden("penalty_windows")
    for w in meta["windows"]:
        out, _, _ = _run_sampler_on_final_logits(t["logits"], t["generated"],
                                                 dict(temperature=0.0, repetition_penalty_window=w))
        assert torch.equal(out, t[f"greedy{w}"]), w


def test_sampler_stochastic_matches_reference_with_same_noise():
    t, meta = load_golden("samplers")
    for i, ps in enumerate(meta["params"]):
        out, _, _ = _run_sampler_on_final_logits(t["logits"], t["generated"], ps, noise=t[f"q{i}"])
        agree = (out == t[f"out{i}"]).float().mean().item()
        assert agree == 1.0, (ps, agree)


def test_sampler_noise_is_exponential():
    # counter-hash exponential race: a uniform distribution must be sampled uniformly
    logits = torch.zeros(64, 9, 1026)
    logits[..., 1024:] = -torch.inf
    gen = torch.full((64, 9, 2), 1025)
    out, _, _ = _run_sampler_on_final_logits(logits, gen, dict(temperature=1.0, repetition_penalty=1.0))
    counts = torch.bincount(out.flatten(), minlength=1024).float()
    assert out.max() < 1024
    assert counts.max() <= 8  # 576 draws over 1024 tokens
    assert len(set(out.flatten().tolist())) > 350


def test_sample_from_logits_v1025_mask_tokens_penalise_eos():
    """Unpadded heads (V = 1025): the reference clamps the penalty window to V - 1 = 1024 (sampling.py:111), so a
    mask token (1025) in the window penalises the EOS column. Greedy, against oracle.zonos_cpu's restatement."""
    from zonos_vibes_amd.sampling import sample_from_logits
    g = torch.Generator().manual_seed(5)
    logits = torch.randn(4, 9, 1025, generator=g)
    logits[..., 1024] = logits.max(dim=-1).values + 0.5  # EOS wins unless it is penalised
    gen = torch.randint(0, 1024, (4, 9, 3), generator=g)
    gen[:2, :, -1] = 1025  # mask tokens in the window of batch rows 0, 1
    ref = oz.repetition_penalty(logits, gen, 3.0, 2).argmax(dim=-1)
    out = sample_from_logits(logits.to(DEV), temperature=0.0, generated_tokens=gen.to(DEV), repetition_penalty=3.0,
                             repetition_penalty_window=2)
    assert torch.equal(out.squeeze(-1).cpu(), ref)
    assert (ref[:2] != 1024).any() and (ref[2:] == 1024).all()


def test_delay_pattern_init_and_revert():
    L = _lib()
    t, _ = load_golden("delay_pattern")
    sl, st, delayed, _ = _slots(2, 32)
    codes = t["codes"]  # [2, 9, 12] with -1 for the last 3
    for s in range(2):
        pre = codes[s, :, :9].to(DEV, torch.int32).contiguous()
        L.check(L.lib().zmi_delay_init(ctypes.byref(sl), s, pre.data_ptr(), 9, 12 + 9, stream_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(delayed[:, :, :21].cpu().long(), t["delayed"])
    out = torch.zeros(9, 12, dtype=torch.int64, device=DEV)
    L.check(L.lib().zmi_delay_revert(ctypes.byref(sl), 0, out.data_ptr(), 12, stream_ptr()))
    torch.cuda.synchronize()
    ref = t["reverted"][0].clone()
    ref[ref >= 1024] = 0
    assert torch.equal(out.cpu(), ref)


def test_fill_uniform_matches_numpy():
    L = _lib()
    from zonos_vibes_amd import synthetic as syn
    sp = syn.Spec("backbone.layers.0.mixer.in_proj.weight", (37, 129), "bf16", 0.0346, 0.5)
    t = torch.empty(sp.shape, dtype=torch.bfloat16, device=DEV)
    L.check(L.lib().zmi_fill_uniform(t.data_ptr(), sp.numel, syn.tensor_key(7, sp.name), sp.scale, sp.offset, 0,
                                     stream_ptr()))
    ref = syn.materialize_np(sp, 7)
    assert (t.cpu().view(torch.int16).numpy().view("uint16") == ref).all()
