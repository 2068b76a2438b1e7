"""The K-split pair form of the many-row K = 2048 GEMM (zmi_gemv_rows_pair, csrc/zmi_gemm_pair.hip) against
zmi_gemv_launch: every row bit-identical for every epilogue it takes (reference _torch.py:114-115,147-152,
model.py:100-101), units split across the two K halves, partial last units and tiles, row groups, and the tile
counters left at zero after every launch (MI355X only)."""
import ctypes

import pytest
import torch

from tests.test_gpu_kernels import DEV, pack, rnd, stream_ptr

pytestmark = pytest.mark.gpu


def _lib():
    from zonos_vibes_amd import _lib as L
    return L


def _args(L, Wp, X, n_pad, out, ldo, n_valid, extra=None):
    a = L.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), X.data_ptr(), X.shape[0], n_pad, X.shape[1], X.shape[1]
    a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), ldo, n_valid, 1e-5
    if extra:
        extra(a)
    return a


CASES = {  # name: (N, epilogue, pack mode)
    "qkv": (3072, "qkv", 0), "fc1": (16384, "swiglu", 1), "heads": (9234, "logits", 0),
    "in_proj": (8512, "store", 0), "out_proj": (2048, "residual", 0), "narrow": (136, "f32", 0)}


@pytest.mark.parametrize("M", [17, 40, 128, 322])
@pytest.mark.parametrize("name", list(CASES))
def test_rows_pair_equals_gemv(name, M):
    from zonos_vibes_amd.engine import rope_table
    L = _lib()
    lib = L.lib()
    N, epi, mode = CASES[name]
    K = 2048
    W = rnd(N, K, scale=0.03, seed=40)
    X = rnd(M, K, scale=2.0, seed=41)
    Wp, n_pad = pack(W, mode, n_pad=(N + 15) // 16 * 16 if name == "heads" else None)
    rope = rope_table(128).to(DEV)
    smax = 400
    pos = torch.randint(0, smax, (M,), generator=torch.Generator().manual_seed(42), dtype=torch.int32).to(DEV)
    res = rnd(M, N, scale=4.0, seed=43)
    nbytes = lib.zmi_gemv_rows_pair_bytes(M, n_pad)
    assert nbytes > 0
    work = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
    n_tiles, n_units = (M + 15) // 16, (n_pad // 8 + 15) // 16
    flag_words = n_tiles * n_units

    def run(pair):
        if epi == "f32":
            outs = (torch.zeros(M, N, dtype=torch.float32, device=DEV),)
            code, ldo = L.EPI_F32, N
        elif epi == "store":
            outs = (torch.zeros(M, N, dtype=torch.bfloat16, device=DEV),)
            code, ldo = L.EPI_STORE, N
        elif epi == "swiglu":
            outs = (torch.zeros(M, N // 2, dtype=torch.bfloat16, device=DEV),)
            code, ldo = L.EPI_SWIGLU, N // 2
        elif epi == "residual":
            outs = (res.clone(),)
            code, ldo = L.EPI_RESIDUAL, N
        elif epi == "logits":
            outs = (torch.zeros(M, 9, 1026, dtype=torch.float32, device=DEV),)
            code, ldo = L.EPI_LOGITS, 0
        else:
            outs = (torch.zeros(M, 2048, dtype=torch.bfloat16, device=DEV),
                    torch.zeros(M, 4, smax, 128, dtype=torch.bfloat16, device=DEV),
                    torch.zeros(M, 4, 128, smax, dtype=torch.bfloat16, device=DEV))
            code, ldo = L.EPI_QKV, 2048
        row_kv = torch.arange(M, dtype=torch.int32, device=DEV)

        def extra(a):
            if epi == "qkv":
                a.row_kv, a.row_pos = row_kv.data_ptr(), pos.data_ptr()
                a.k_cache, a.v_cache = outs[1].data_ptr(), outs[2].data_ptr()
                a.smax, a.hq, a.hkv, a.hd, a.rope = smax, 16, 4, 128, rope.data_ptr()
        a = _args(L, Wp, X, n_pad, outs[0], ldo, N, extra)
        if pair:
            L.check(lib.zmi_gemv_rows_pair(ctypes.byref(a), code, work.data_ptr(), work.numel(), stream_ptr()),
                    "rows_pair")
        else:
            L.check(lib.zmi_gemv_launch(ctypes.byref(a), code, stream_ptr()), "gemv")
        torch.cuda.synchronize()
        return outs

    ref = run(False)
    for rep in range(2):  # the second launch finds the counters the first left at zero
        got = run(True)
        assert int(work[:flag_words * 4].view(torch.int32).abs().sum()) == 0, (name, M, rep)
        for r, g in zip(ref, got):
            assert torch.equal(g, r), (name, M, rep)


def test_rows_pair_rejects_bad_args():
    L = _lib()
    lib = L.lib()
    W = rnd(256, 2048, scale=0.03, seed=44)
    X = rnd(40, 2048, seed=45)
    Wp, n_pad = pack(W)
    out = torch.zeros(40, 256, dtype=torch.float32, device=DEV)
    small = torch.zeros(16, dtype=torch.uint8, device=DEV)
    a = _args(L, Wp, X, n_pad, out, 256, 256)
    assert lib.zmi_gemv_rows_pair(ctypes.byref(a), L.EPI_F32, small.data_ptr(), small.numel(), stream_ptr()) != 0
    a.K = 1024
    work = torch.zeros(lib.zmi_gemv_rows_pair_bytes(40, 256), dtype=torch.uint8, device=DEV)
    assert lib.zmi_gemv_rows_pair(ctypes.byref(a), L.EPI_F32, work.data_ptr(), work.numel(), stream_ptr()) != 0
