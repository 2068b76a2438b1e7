"""The fused attention + out_proj + fc1 decode launch (zmi_attn_ffn_block) against the same ops as separate
launches (zmi_attention over the KV cache, zmi_gemv_launch EPI_RESIDUAL, then the LayerNorm'd fc1 with
EPI_SWIGLU): the attention rows, the new residual rows x and the FFN hidden rows h must be bit-identical,
at chunk and 512-key block edges, position 0, the last covered position, inactive rows, and over hand-off
granules holding stale tags of earlier steps (as in a running decode). The separate path is pinned against
the oracle / fp32 SDPA in test_gpu_kernels.py."""
import ctypes

import pytest
import torch

from tests.test_gpu_kernels import DEV, _lib, pack, rnd, stream_ptr

from zonos_vibes_amd import _lib as _zl  # noqa: E402

# a diagnostic form (include/zonos_diag.h): tested when libzonos_diag.so is built (`build --diag`)
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not _zl.diag_available(), reason="libzonos_diag.so not built")]

D, F, H, HKV, HD = 2048, 8192, 16, 4, 128


def _gemv_args(Wp, X, M, N, ldx, out, ldo, ln=None, row_pos=None):
    L = _lib()
    a = L.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx = Wp.data_ptr(), X.data_ptr(), M, N, D, ldx
    a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), ldo, N, 1e-5
    if ln is not None:
        a.ln_w, a.ln_b = ln[0].data_ptr(), ln[1].data_ptr()
    if row_pos is not None:
        a.row_pos = row_pos.data_ptr()
    return a


def _stale(n):
    return torch.randint(0, 1 << 30, (n,), device=DEV) | (torch.randint(1 << 20, 1 << 30, (n,), device=DEV) << 32)


@pytest.mark.parametrize("positions", [(591, 591), (0,), (5, -1), (1023, 1022), (127, 128), (511, 512), (-1, 900)])
def test_attn_ffn_block_bit_identical_to_separate_launches(positions):
    L = _lib()
    if torch.cuda.get_device_properties(0).multi_processor_count < 256:
        pytest.skip("zmi_attn_ffn_block needs 256 CUs")
    M, smax = len(positions), 1032
    assert max(positions) <= L.diag().zmi_attn_ffn_max_pos()
    q = rnd(M, H * HD, scale=1.0, seed=80)
    kc = rnd(M, HKV, smax, HD, seed=81)
    vt = rnd(M, HKV, HD, smax, seed=82)
    Wo, Wf = rnd(D, D, scale=0.03, seed=83), rnd(2 * F, D, scale=0.03, seed=84)
    Po, Pf = pack(Wo)[0], pack(Wf, mode=1)[0]
    x0 = rnd(M, D, scale=2.0, seed=85)
    ln = ((rnd(D, scale=0.1, seed=86) + 1).contiguous(), rnd(D, scale=0.02, seed=87))
    attn0 = rnd(M, D, scale=1.0, seed=88)  # what the attention rows buffer holds before (inactive rows keep it)
    row_pos = torch.tensor(positions, dtype=torch.int32, device=DEV)
    live = [i for i, p in enumerate(positions) if p >= 0]

    # separate launches
    attn_s = attn0.clone()
    work = torch.zeros(L.lib().zmi_attention_work_bytes(M, H, HKV, HD, smax - 1), dtype=torch.uint8, device=DEV)
    nf = L.lib().zmi_attention_partial_floats(M, H, HKV, HD, smax - 1)
    po = torch.zeros(nf, dtype=torch.float32, device=DEV)
    plm = torch.zeros(nf // HD * 2, dtype=torch.float32, device=DEV)
    L.check(L.lib().zmi_attention_variant(q.data_ptr(), H * HD, kc.data_ptr(), vt.data_ptr(), None, row_pos.data_ptr(),
                                          M, H, HKV, HD, smax, smax - 1, attn_s.data_ptr(), H * HD, po.data_ptr(),
                                          plm.data_ptr(), work.data_ptr(), 1, stream_ptr()), "attention")
    xs, hs = x0.clone(), torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
    a = _gemv_args(Po, attn_s, M, D, D, xs, D)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(a), L.EPI_RESIDUAL, stream_ptr()))
    b = _gemv_args(Pf, xs, M, 2 * F, D, hs, F, ln=ln)
    L.check(L.lib().zmi_gemv_launch(ctypes.byref(b), L.EPI_SWIGLU, stream_ptr()))

    # fused, three times at the same positions over granules holding stale tags
    qa = L.GemvArgs()
    qa.M, qa.K, qa.out, qa.ldo = M, D, q.data_ptr(), H * HD
    qa.row_pos, qa.k_cache, qa.v_cache = row_pos.data_ptr(), kc.data_ptr(), vt.data_ptr()
    qa.smax, qa.hq, qa.hkv, qa.hd = smax, H, HKV, HD
    xg = _stale(L.lib().zmi_attn_block_gran_words(M, HKV))
    og = _stale(L.diag().zmi_attn_ffn_gran_words(M))
    rg = _stale(L.diag().zmi_attn_ffn_gran_words(M))
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    for rep in range(3):
        attn_f = attn0.clone()
        xf, hf = x0.clone(), torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
        a = _gemv_args(Po, attn_f, M, D, D, xf, D, row_pos=row_pos)
        b = _gemv_args(Pf, xf, M, 2 * F, D, hf, F, ln=ln)
        L.check(L.diag().zmi_attn_ffn_block(ctypes.byref(qa), ctypes.byref(a), ctypes.byref(b), xg.data_ptr(),
                                           og.data_ptr(), rg.data_ptr(), err.data_ptr(), attn_f.data_ptr(), H * HD,
                                           stream_ptr()), "attn_ffn_block")
        torch.cuda.synchronize()
        assert int(err[0].item()) == 0, "a hand-off wait gave up"
        assert torch.equal(attn_f, attn_s), rep
        assert torch.equal(xf, xs), rep
        assert torch.equal(hf[live], hs[live]), rep
