"""The split-K fc2 / out_proj GEMM (zmi_gemv_splitk: one workgroup per 64-column block, K segment -- 8 x 1024
for K = 8192, 4 x 1024 for the hybrid's K = 4096 Mamba2 out_proj, 4 x 512 for K = 2048 -- and row group, fp32
segment sums, a reduce launch adding them in K order + the residual / store epilogue) against zmi_gemv_launch's
GEMV for the same op: bit-identical for row counts on and off the 16-row tile, across the GEMV's own launch forms
at those counts and across row groupings (a row's result may not depend on the batch it is computed in)."""
import ctypes

import pytest
import torch

from tests.test_gpu_kernels import DEV, _lib, pack, rnd, stream_ptr

pytestmark = pytest.mark.gpu

D, F = 2048, 8192


@pytest.mark.parametrize("stage", [1, 0])  # ZMI_OPT_SPLITK_STAGE: several 16-row tiles per LDS stage buffer
@pytest.mark.parametrize("rows_opt", [1, 3])  # ZMI_OPT_GEMM_ROWS bit 1: the dense-pair MFMA form
@pytest.mark.parametrize("wgs", [256, 0, 1024])
@pytest.mark.parametrize("K", [F, 4096, D])
@pytest.mark.parametrize("M", [1, 16, 17, 64, 65, 128, 322])
def test_splitk_bit_identical_to_gemv(M, K, wgs, rows_opt, stage):
    L = _lib()
    epi = L.EPI_STORE if K == 4096 else L.EPI_RESIDUAL
    W = rnd(D, K, scale=0.03, seed=70)
    Wp = pack(W)[0]
    h = rnd(M, K, scale=1.0, seed=71)
    x0 = rnd(M, D, scale=2.0, seed=72)

    def args(out):
        a = L.GemvArgs()
        a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), h.data_ptr(), M, D, K, K
        a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), D, D, 1e-5
        return a

    ref = x0.clone()
    a = args(ref)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(a), epi, stream_ptr()))
    got = x0.clone()
    nf = L.lib().zmi_gemv_splitk_floats(M, D)
    part = torch.full((nf,), float("nan"), dtype=torch.float32, device=DEV)
    a = args(got)
    knobs = {L.OPT_SPLITK_WGS: wgs, L.OPT_GEMM_ROWS: rows_opt, L.OPT_SPLITK_STAGE: stage}
    old = {k: L.lib().zmi_get_option(k) for k in knobs}
    for k, v in knobs.items():
        L.lib().zmi_set_option(k, v)
    try:
        L.check(L.lib().zmi_gemv_splitk(ctypes.byref(a), epi, part.data_ptr(), nf, stream_ptr()), "splitk")
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            L.lib().zmi_set_option(k, v)
    assert torch.equal(got, ref), (got != ref).nonzero()[:4].tolist()


@pytest.mark.parametrize("K", [F, D])
@pytest.mark.parametrize("M", [16, 33, 128])
def test_splitk_fused_layernorm_bit_identical(M, K):
    """zmi_gemv_splitk_ln: the reduce also writes LayerNorm(new rows) -- equal to the GEMV followed by
    zmi_layernorm_rows (the next op's pre-pass it replaces)."""
    L = _lib()
    W = rnd(D, K, scale=0.03, seed=73)
    Wp = pack(W)[0]
    h = rnd(M, K, scale=1.0, seed=74)
    x0 = rnd(M, D, scale=2.0, seed=75)
    lw, lb = (rnd(D, scale=0.1, seed=76) + 1).contiguous(), rnd(D, scale=0.02, seed=77)

    def args(out):
        a = L.GemvArgs()
        a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), h.data_ptr(), M, D, K, K
        a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), D, D, 1e-5
        return a

    ref = x0.clone()
    a = args(ref)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(a), L.EPI_RESIDUAL, stream_ptr()))
    ref_n = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    L.check(L.lib().zmi_layernorm_rows(ref.data_ptr(), D, M, D, lw.data_ptr(), lb.data_ptr(), 1e-5, ref_n.data_ptr(), D,
                                       stream_ptr()))
    got = x0.clone()
    got_n = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    nf = L.lib().zmi_gemv_splitk_floats(M, D)
    part = torch.full((nf,), float("nan"), dtype=torch.float32, device=DEV)
    a = args(got)
    L.check(L.lib().zmi_gemv_splitk_ln(ctypes.byref(a), L.EPI_RESIDUAL, part.data_ptr(), nf, lw.data_ptr(), lb.data_ptr(),
                                       1e-5, got_n.data_ptr(), D, stream_ptr()), "splitk_ln")
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert torch.equal(got_n, ref_n), (got_n != ref_n).nonzero()[:4].tolist()


def test_engine_splitk_and_attention_prefetch_bit_identical():
    """Engine level: 8 utterances through generate_batch on 8 slots -- the prefill's out_proj / fc2
    at M = 2 S rows and the 16-row decode steps take the split-K GEMMs (with the fused LayerNorm) and the chunked
    attention launch with its prefetch role by default -- against the same run with split-K off (the GEMV plan)
    and with the prefetch role off: identical codes and identical final logits."""
    from zonos_vibes_amd.config import transformer_config
    from zonos_vibes_amd.model import Zonos
    cfg = transformer_config(2048, 3, 16, 4, 8192)
    lcs = [40, 33, 57, 40, 21, 64, 48, 30]
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_slots=8, max_seqlen=64 + 40 + 16, max_prefill=64 + 8)
    e = m.engine
    g = torch.Generator().manual_seed(5)
    conds = [(torch.randn(2, lc, 2048, generator=g) * 0.5).to(torch.bfloat16).to(DEV) for lc in lcs]

    def run(**opts):
        for k, v in opts.items():
            setattr(e, k, v)
        e._build_plan()
        out = m.generate_batch(conds, max_new_tokens=40, sampling_params=dict(temperature=0.0), seeds=list(range(8)),
                               max_slots=8)
        return [c.cpu() for c in out], e.logits.clone()

    ref_codes, ref_logits = run(attn_prefetch_blocks=256)
    assert e._use_splitk(*e._gemv(e.w["layers"][0]["fc2"], e.h, 16, 2048, 8192, _lib().EPI_RESIDUAL, e.x, 2048))
    for opts in (dict(splitk_rows=0, splitk_o_rows=0), dict(splitk_rows=16, splitk_o_rows=16, attn_prefetch_blocks=0)):
        codes, logits = run(**opts)
        assert all(torch.equal(a, b) for a, b in zip(codes, ref_codes)), opts
        assert torch.equal(logits, ref_logits), opts
