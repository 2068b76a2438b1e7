"""The persistent FFN decode engine (zmi_ffn_engine: out_proj + residual, norm2, fc1 + SwiGLU, fc2 + residual
in one launch of 256 workgroups) against the same ops as separate zmi_gemv_launch calls: the new residual rows
and the SwiGLU rows must be bit-identical (reference zonos/backbone/_torch.py:100-101, 147-152)."""
import ctypes

import pytest
import torch

from tests.test_gpu_kernels import DEV, _lib, pack, rnd, stream_ptr

from zonos_vibes_amd import _lib as _zl  # noqa: E402

# a diagnostic form (include/zonos_diag.h): tested when libzonos_diag.so is built (`build --diag`)
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not _zl.diag_available(), reason="libzonos_diag.so not built")]

D, F = 2048, 8192


def _gemv(L, Wp, X, M, N, K, out, ldo, epi, ln=None):
    a = L.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), X.data_ptr(), M, N, K, K
    a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), ldo, N, 1e-5
    if ln is not None:
        a.ln_w, a.ln_b = ln[0].data_ptr(), ln[1].data_ptr()
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(a), epi, stream_ptr()), "gemv")


def _weights(seed):
    Wo, Wf, W2 = rnd(D, D, scale=0.03, seed=seed), rnd(2 * F, D, scale=0.03, seed=seed + 1), \
        rnd(D, F, scale=0.02, seed=seed + 2)
    ln = ((rnd(D, scale=0.1, seed=seed + 3) + 1).contiguous(), rnd(D, scale=0.02, seed=seed + 4))
    return pack(Wo)[0], pack(Wf, mode=1)[0], pack(W2)[0], ln


def _engine(L, Po, Pf, P2, ln, attn, x, h, row_pos, gran, err, diag=None):
    e = L.FfnEngineArgs()
    e.w_out, e.w_fc1, e.w_fc2 = Po.data_ptr(), Pf.data_ptr(), P2.data_ptr()
    e.ln_w, e.ln_b, e.eps = ln[0].data_ptr(), ln[1].data_ptr(), 1e-5
    e.M = x.shape[0]
    e.attn, e.x, e.h = attn.data_ptr(), x.data_ptr(), (h.data_ptr() if h is not None else None)
    e.ld_attn, e.ldx, e.ldh = attn.shape[1], x.shape[1], F
    e.row_pos, e.gran, e.err = row_pos.data_ptr(), gran.data_ptr(), err.data_ptr()
    e.diag = diag.data_ptr() if diag is not None else None
    L.check(L.diag().zmi_ffn_engine(ctypes.byref(e), stream_ptr()), "ffn_engine")


@pytest.mark.parametrize("positions", [(591, 591), (0,), (1023, 1023), (5000, 5000)])
def test_ffn_engine_bit_identical_to_separate_launches(positions):
    L = _lib()
    if torch.cuda.get_device_properties(0).multi_processor_count < 256:
        pytest.skip("zmi_ffn_engine needs 256 CUs")
    M = len(positions)
    Po, Pf, P2, ln = _weights(100)
    attn = rnd(M, D, scale=1.0, seed=110)
    x0 = rnd(M, D, scale=2.0, seed=111)
    row_pos = torch.tensor(positions, dtype=torch.int32, device=DEV)
    # separate launches: out_proj (residual), fc1 (norm2 prologue, SwiGLU), fc2 (residual)
    xs, hs = x0.clone(), torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
    _gemv(L, Po, attn, M, D, D, xs, D, L.EPI_RESIDUAL)
    _gemv(L, Pf, xs, M, 2 * F, D, hs, F, L.EPI_SWIGLU, ln=ln)
    _gemv(L, P2, hs, M, D, F, xs, D, L.EPI_RESIDUAL)
    # engine: three launches at the same position over granules holding stale tags, then at the next position
    gran = torch.randint(0, 1 << 30, (L.diag().zmi_ffn_engine_gran_words(M),), device=DEV, dtype=torch.int64)
    gran |= torch.randint(1 << 20, 1 << 30, gran.shape, device=DEV) << 32
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    for rep in range(3):
        xf, hf = x0.clone(), torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
        _engine(L, Po, Pf, P2, ln, attn, xf, hf, row_pos, gran, err)
        torch.cuda.synchronize()
        assert int(err[0].item()) == 0, "a hand-off wait gave up"
        assert torch.equal(hf, hs), rep
        assert torch.equal(xf, xs), rep
    xf = x0.clone()
    _engine(L, Po, Pf, P2, ln, attn, xf, None, row_pos + 1, gran, err)
    torch.cuda.synchronize()
    assert int(err[0].item()) == 0
    assert torch.equal(xf, xs)


def test_ffn_engine_layer_chain():
    """Several layers back to back (each its own weights and granule area), as in a decode step."""
    L = _lib()
    if torch.cuda.get_device_properties(0).multi_processor_count < 256:
        pytest.skip("zmi_ffn_engine needs 256 CUs")
    M, NL = 2, 3
    layers = [_weights(200 + 10 * i) for i in range(NL)]
    attn = [rnd(M, D, scale=1.0, seed=300 + i) for i in range(NL)]
    x0 = rnd(M, D, scale=2.0, seed=310)
    row_pos = torch.tensor([77, 77], dtype=torch.int32, device=DEV)
    xs, hs = x0.clone(), torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
    for (Po, Pf, P2, ln), at in zip(layers, attn):
        _gemv(L, Po, at, M, D, D, xs, D, L.EPI_RESIDUAL)
        _gemv(L, Pf, xs, M, 2 * F, D, hs, F, L.EPI_SWIGLU, ln=ln)
        _gemv(L, P2, hs, M, D, F, xs, D, L.EPI_RESIDUAL)
    words = L.diag().zmi_ffn_engine_gran_words(M)
    gran = torch.zeros(NL, words, dtype=torch.int64, device=DEV)
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    xf = x0.clone()
    for i, ((Po, Pf, P2, ln), at) in enumerate(zip(layers, attn)):
        _engine(L, Po, Pf, P2, ln, at, xf, None, row_pos, gran[i], err)
    torch.cuda.synchronize()
    assert int(err[0].item()) == 0
    assert torch.equal(xf, xs)
