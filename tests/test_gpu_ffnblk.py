"""The fused out_proj + fc1 decode launch (zmi_ffn_block) against the same two ops as separate launches
(zmi_gemv_launch EPI_RESIDUAL on the residual rows, then the LayerNorm'd fc1 with EPI_SWIGLU): the new
residual rows x and the FFN hidden rows h must be bit-identical, for 1 .. 16 rows, inactive rows, and
hand-off granules holding stale tags of earlier steps (as in a running decode)."""
import ctypes

import pytest
import torch

from tests.test_gpu_kernels import DEV, _lib, pack, rnd, stream_ptr

from zonos_vibes_amd import _lib as _zl  # noqa: E402

# a diagnostic form (include/zonos_diag.h): tested when libzonos_diag.so is built (`build --diag`)
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not _zl.diag_available(), reason="libzonos_diag.so not built")]

D, F = 2048, 8192


def _args(Wp, X, M, N, ldx, out, ldo, ln=None, row_pos=None):
    L = _lib()
    a = L.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), X.data_ptr(), M, N, D, ldx
    a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), ldo, N, 1e-5
    if ln is not None:
        a.ln_w, a.ln_b = ln[0].data_ptr(), ln[1].data_ptr()
    if row_pos is not None:
        a.row_pos = row_pos.data_ptr()
    return a


@pytest.mark.parametrize("positions", [(591, 591), (0,), (5, -1, 300, 301, 63, 64, 700, -1, 1000, 1001, 31, 32, 255,
                                                              256, 900, 17), (7, 8, 9, 10, 11)])
def test_ffn_block_bit_identical_to_separate_launches(positions):
    L = _lib()
    if torch.cuda.get_device_properties(0).multi_processor_count < 256:
        pytest.skip("zmi_ffn_block needs 256 CUs")
    M = len(positions)
    Wo, Wf = rnd(D, D, scale=0.03, seed=90), rnd(2 * F, D, scale=0.03, seed=91)
    Po, Pf = pack(Wo)[0], pack(Wf, mode=1)[0]
    attn = rnd(M, D, scale=1.0, seed=92)
    x0 = rnd(M, D, scale=2.0, seed=93)
    ln = ((rnd(D, scale=0.1, seed=94) + 1).contiguous(), rnd(D, scale=0.02, seed=95))
    row_pos = torch.tensor(positions, dtype=torch.int32, device=DEV)
    live = [i for i, p in enumerate(positions) if p >= 0]
    # separate launches
    xs, hs = x0.clone(), torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
    a = _args(Po, attn, M, D, D, xs, D)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(a), L.EPI_RESIDUAL, stream_ptr()))
    b = _args(Pf, xs, M, 2 * F, D, hs, F, ln=ln)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(b), L.EPI_SWIGLU, stream_ptr()))
    # fused, three times at the same positions over granules holding stale tags
    gran = torch.zeros(L.diag().zmi_ffn_block_gran_words(M), dtype=torch.int64, device=DEV)
    gran.copy_(torch.randint(0, 1 << 30, gran.shape, device=DEV) |
               (torch.randint(1 << 20, 1 << 30, gran.shape, device=DEV) << 32))
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    for rep in range(3):
        xf, hf = x0.clone(), torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
        a = _args(Po, attn, M, D, D, xf, D, row_pos=row_pos)
        b = _args(Pf, xf, M, 2 * F, D, hf, F, ln=ln)
        L.check(L.diag().zmi_ffn_block(ctypes.byref(a), ctypes.byref(b), gran.data_ptr(), err.data_ptr(),
                                      stream_ptr()), "ffn_block")
        torch.cuda.synchronize()
        assert int(err[0].item()) == 0, "a hand-off wait gave up"
        assert torch.equal(xf, xs), rep
        assert torch.equal(hf[live], hs[live]), rep
