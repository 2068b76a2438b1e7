"""The fused decode block (zmi_attn_block: QKV projection + attention in ONE launch) against the
same two ops as separate launches (zmi_gemv_launch EPI_QKV, then zmi_attention): q, the K / V
cache writes and the attention output must be bit-identical, for any row count up to 16, mixed
positions (chunk and 512-key block edges, position 0, the last covered position) and inactive rows.
The separate path is itself pinned against the oracle / fp32 SDPA in test_gpu_kernels.py."""
import ctypes

import pytest
import torch

from tests.test_gpu_kernels import DEV, _check_attention, _lib, pack, rnd, stream_ptr

pytestmark = pytest.mark.gpu

D, H, HKV, HD = 2048, 16, 4, 128
QKV_N = (H + 2 * HKV) * HD


def _setup(positions, smax, seed):
    from zonos_vibes_amd.engine import rope_table
    R = len(positions)
    W = rnd(QKV_N, D, scale=0.03, seed=seed)
    X = rnd(R, D, scale=2.0, seed=seed + 1)
    lw, lb = rnd(D, scale=0.1, seed=seed + 2) + 1, rnd(D, scale=0.02, seed=seed + 3)
    kc = rnd(R, HKV, smax, HD, seed=seed + 4)
    vt = rnd(R, HKV, HD, smax, seed=seed + 5)
    return dict(W=pack(W), X=X, ln=(lw.contiguous(), lb.contiguous()), kc=kc, vt=vt, rope=rope_table(HD).to(DEV),
                row_kv=torch.arange(R, dtype=torch.int32, device=DEV),
                row_pos=torch.tensor(positions, dtype=torch.int32, device=DEV), smax=smax, R=R)


def _args(st, q, kc, vt):
    L = _lib()
    (Wp, n_pad) = st["W"]
    a = L.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), st["X"].data_ptr(), st["R"], n_pad, D, D
    a.ln_w, a.ln_b, a.eps = st["ln"][0].data_ptr(), st["ln"][1].data_ptr(), 1e-5
    a.out, a.ldo, a.n_valid = q.data_ptr(), H * HD, QKV_N
    a.row_kv, a.row_pos, a.k_cache, a.v_cache = st["row_kv"].data_ptr(), st["row_pos"].data_ptr(), kc.data_ptr(), \
        vt.data_ptr()
    a.smax, a.hq, a.hkv, a.hd, a.rope = st["smax"], H, HKV, HD, st["rope"].data_ptr()
    return a


def _separate(st):
    L = _lib()
    R, smax = st["R"], st["smax"]
    q = torch.zeros(R, H * HD, dtype=torch.bfloat16, device=DEV)
    kc, vt = st["kc"].clone(), st["vt"].clone()
    a = _args(st, q, kc, vt)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(a), L.EPI_QKV, stream_ptr()), "gemv")
    out = torch.zeros(R, H * HD, dtype=torch.bfloat16, device=DEV)
    work = torch.zeros(L.lib().zmi_attention_work_bytes(R, H, HKV, HD, smax - 1), dtype=torch.uint8, device=DEV)
    nf = L.lib().zmi_attention_partial_floats(R, H, HKV, HD, smax - 1)
    po = torch.zeros(nf, dtype=torch.float32, device=DEV)
    plm = torch.zeros(nf // HD * 2, dtype=torch.float32, device=DEV)
    L.check(L.lib().zmi_attention_variant(q.data_ptr(), H * HD, kc.data_ptr(), vt.data_ptr(), None,
                                          st["row_pos"].data_ptr(), R, H, HKV, HD, smax, smax - 1, out.data_ptr(),
                                          H * HD, po.data_ptr(), plm.data_ptr(), work.data_ptr(), 1, stream_ptr()))
    torch.cuda.synchronize()
    return q, kc, vt, out


def _fused(st, slices, reps=1):
    L = _lib()
    R = st["R"]
    q = torch.zeros(R, H * HD, dtype=torch.bfloat16, device=DEV)
    kc, vt = st["kc"].clone(), st["vt"].clone()
    a = _args(st, q, kc, vt)
    # hand-off granules hold stale tags of "earlier steps" (every tag except position + 1 of the row),
    # as they do in a running decode
    gran = torch.zeros(L.lib().zmi_attn_block_gran_words(R, HKV), dtype=torch.int64, device=DEV)
    stale = torch.randint(0, 1 << 30, gran.shape, device=DEV)
    gran.copy_(stale | ((torch.randint(1 << 20, 1 << 30, gran.shape, device=DEV)) << 32))
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    out = torch.zeros(R, H * HD, dtype=torch.bfloat16, device=DEV)
    for _ in range(reps):  # a repeated launch at the same positions reads its own (equal) granules
        L.check(L.lib().zmi_attn_block(ctypes.byref(a), gran.data_ptr(), err.data_ptr(), out.data_ptr(), H * HD,
                                       slices, stream_ptr()), "attn_block")
    torch.cuda.synchronize()
    assert int(err[0].item()) == 0, "a wait for a hand-off gave up"
    return q, kc, vt, out


SELF, SPLIT = 256, 512  # zmi_attn_block slices flags: self-scoring / chunk-split forms (positions < 1024)


@pytest.mark.parametrize("positions", [
    (591, 592),                                    # C2 mean position, one slot
    (0, 1),                                        # the first key comes from this launch only
    (127, 128, 511, 512, 1030, 1279),              # chunk / block edges and the last covered position
    (5, -1, 300, 301, 63, 64, 700, -1, 1000, 1001, 31, 32, 255, 256, 900, 17),  # 16 rows, inactive rows
])
@pytest.mark.parametrize("slices", [4, 8, 4 | SELF, 8 | SELF, 8 | SPLIT])
@pytest.mark.parametrize("smax", [1280, 2056])
def test_attn_block_bit_identical_to_separate_launches(positions, slices, smax):
    if slices & (SELF | SPLIT):  # these forms reach position 1023: keep the edges inside it
        positions = tuple(p if p < 1024 else p - 256 for p in positions) + ((1023,) if len(positions) < 16 else ())
    assert max(positions) <= _lib().lib().zmi_attn_block_max_pos(slices)
    st = _setup(positions, smax, seed=70)
    ref = _separate(st)
    got = _fused(st, slices, reps=3)
    live = [i for i, p in enumerate(positions) if p >= 0]
    for name, r, g in zip(("q", "k_cache", "v_cache"), ref[:3], got[:3]):
        assert torch.equal(r, g), name
    assert torch.equal(ref[3][live], got[3][live]), "attention output"
    # and the output is the reference attention of the projected q / K / V
    pick = live[:3]
    _check_attention(got[3][pick], got[0][pick], got[1][pick], got[2][pick].transpose(-1, -2).contiguous(),
                     [positions[i] for i in pick])


@pytest.mark.parametrize("positions", [
    (1024, 1025),                                   # just past the 8-chunk form: one batch-1 step
    (0, 1, 1535, 1536, 2047, 2048, 2559, 3071),    # block edges of the wide form and its last position
    (1200, 1201),
    (3000, 2999),
])
@pytest.mark.parametrize("smax", [3072, 3200])
def test_attn_block_wide_split_bit_identical_to_separate_launches(positions, smax):
    """The 24-chunk split form (batch-1 decode steps past the 8-chunk reach, up to position 3071): q, the KV
    cache writes and the attention output bit-identical to the QKV GEMV + chunked attention launches."""
    slices = 24 | SPLIT
    assert max(positions) <= _lib().lib().zmi_attn_block_max_pos(slices) == 3071
    st = _setup(positions, smax, seed=72)
    ref = _separate(st)
    got = _fused(st, slices, reps=3)
    for name, r, g in zip(("q", "k_cache", "v_cache"), ref[:3], got[:3]):
        assert torch.equal(r, g), name
    assert torch.equal(ref[3], got[3]), "attention output"
    _check_attention(got[3][:2], got[0][:2], got[1][:2], got[2][:2].transpose(-1, -2).contiguous(), list(positions[:2]))


@pytest.mark.parametrize("slices", [8, 8 | SELF, 8 | SPLIT, 24 | SPLIT])
def test_attn_block_refuses_positions_past_its_reach(slices):
    """A row past the form's last position sets the error word instead of reading past its K / V reach."""
    L = _lib()
    last = L.lib().zmi_attn_block_max_pos(slices)
    st = _setup((100, last + 1), 2056, seed=71)
    q = torch.zeros(2, H * HD, dtype=torch.bfloat16, device=DEV)
    kc, vt = st["kc"].clone(), st["vt"].clone()
    a = _args(st, q, kc, vt)
    gran = torch.zeros(L.lib().zmi_attn_block_gran_words(2, HKV), dtype=torch.int64, device=DEV)
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    out = torch.zeros(2, H * HD, dtype=torch.bfloat16, device=DEV)
    L.check(L.lib().zmi_attn_block(ctypes.byref(a), gran.data_ptr(), err.data_ptr(), out.data_ptr(), H * HD,
                                   slices, stream_ptr()), "attn_block")
    torch.cuda.synchronize()
    assert int(err[0].item()) != 0


@pytest.mark.parametrize("positions,chunks", [
    ((591, 592), 8),                                 # C2 mean position, one slot
    ((0, 1), 8),
    ((127, 128, 511, 512, 900, 1023), 8),            # chunk / block edges and the form's last position
    ((5, -1, 300, 301, 63, 64, 700, 1000), 8),       # 8 rows (the fused forms' default limit), an inactive row
    ((5, -1, 300, 301, 63, 64, 700, -1, 1000, 1001, 31, 32, 255, 256, 900, 17), 8),  # 16 rows
    ((1024, 1025), 24),                              # the 24-chunk form: batch-1 steps past the 8-chunk reach
    ((1161, 1162), 24),
    ((2661, -1), 24),
    ((3071, 2047, 1535, 1536), 24),                  # the form's last position, block edges
])
def test_attn_block_oproj_bit_identical_to_separate_launches(positions, chunks):
    """zmi_attn_block_oproj (a chunk-split form, 8 or 24 chunk workgroups, with the layer's out_proj GEMV in the same
    launch, its input gathered from the merging workgroups' granules): q, K / V, the attention output and the new
    residual rows bit-identical to the QKV GEMV + attention + out_proj GEMV (EPI_RESIDUAL) launches; run twice (the
    second launch finds its own granules from the first: equal values, equal tags)."""
    L = _lib()
    slices = chunks | SPLIT
    st = _setup(positions, 2056 if chunks == 8 else 3080, seed=80)
    R = st["R"]
    ref_q, ref_k, ref_v, ref_out = _separate(st)
    Wo = pack(rnd(D, H * HD, scale=0.03, seed=81))[0]
    x0 = rnd(R, D, scale=2.0, seed=82)

    def oargs(attn, x):
        o = L.GemvArgs()
        o.W, o.X, o.M, o.N, o.K, o.ldx = Wo.data_ptr(), attn.data_ptr(), R, D, H * HD, H * HD
        o.out, o.ldo, o.n_valid = x.data_ptr(), D, D
        return o

    x_ref = x0.clone()
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(oargs(ref_out, x_ref)), L.EPI_RESIDUAL, stream_ptr()), "out_proj")
    q = torch.zeros(R, H * HD, dtype=torch.bfloat16, device=DEV)
    kc, vt = st["kc"].clone(), st["vt"].clone()
    a = _args(st, q, kc, vt)
    gran = torch.zeros(L.lib().zmi_attn_block_gran_words(R, HKV), dtype=torch.int64, device=DEV)
    gran.copy_(torch.randint(0, 1 << 30, gran.shape, device=DEV) | (torch.randint(1 << 20, 1 << 30, gran.shape,
                                                                                  device=DEV) << 32))
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    out = torch.zeros(R, H * HD, dtype=torch.bfloat16, device=DEV)
    pf = L.Prefetch()
    live = [i for i, p in enumerate(positions) if p >= 0]
    for _ in range(2):
        x = x0.clone()
        L.check(L.lib().zmi_attn_block_oproj(ctypes.byref(a), ctypes.byref(oargs(out, x)), gran.data_ptr(),
                                             err.data_ptr(), out.data_ptr(), H * HD, slices, ctypes.byref(pf),
                                             stream_ptr()), "attn_block_oproj")
        torch.cuda.synchronize()
        assert int(err[0].item()) == 0, "a wait for a hand-off gave up"
        for name, r, g in (("q", ref_q, q), ("k_cache", ref_k, kc), ("v_cache", ref_v, vt)):
            assert torch.equal(r, g), name
        assert torch.equal(ref_out[live], out[live]), "attention output"
        assert torch.equal(x_ref[live], x[live]), "out_proj residual rows"


def test_engine_fused_out_proj_keeps_codes():
    """generate() with out_proj inside the fused block (the default) equals generate() with out_proj as its own
    launch and with separate QKV + attention launches, across the 8-chunk form's reach (positions 900 .. 1100)."""
    from zonos_vibes_amd.config import transformer_config
    from zonos_vibes_amd.model import Zonos
    cfg = transformer_config(2048, 2, 16, 4, 8192)
    lc, n = 900, 200
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_seqlen=lc + n + 16, max_prefill=lc + 8)
    g = torch.Generator().manual_seed(91)
    cond = (torch.randn(2, lc, 2048, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    e = m.engine
    assert any(kd == "attnblk" and it[4] is not None for kd, it in e._plan(2, "split")), "default: out_proj fused"
    out = {}
    for name, opts in (("fused_oproj", dict(attn_block=True, attn_oproj=True)),
                       ("oproj_launch", dict(attn_block=True, attn_oproj=False)),
                       ("separate", dict(attn_block=False, attn_oproj=False))):
        for k, v in opts.items():
            setattr(e, k, v)
        e._build_plan()
        out[name] = m.generate(cond, max_new_tokens=n, sampling_params=dict(temperature=0.0), progress_bar=False,
                               chunk=64)
        e.check_errors()
    assert torch.equal(out["fused_oproj"], out["oproj_launch"])
    assert torch.equal(out["fused_oproj"], out["separate"])
