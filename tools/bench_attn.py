"""Latency probes (HIP events, back-to-back launches) for the decode attention and a 1-block GEMV.

Separates the fixed per-launch chain from the per-chunk / merge cost. One JSON line per probe.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

L = _lib.lib()
dev = "cuda"


def timed(fn, reps=200):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) * 1e3 / reps


def attn(R, pos, smax=1032, H=16, Hkv=4, hd=128):
    q = torch.randn(R, H * hd, device=dev).to(torch.bfloat16)
    kc = torch.randn(R, Hkv, smax, hd, device=dev).to(torch.bfloat16)
    vc = torch.randn(R, Hkv, smax, hd, device=dev).to(torch.bfloat16)
    out = torch.zeros(R, H * hd, device=dev).to(torch.bfloat16)
    rp = torch.full((R,), pos, dtype=torch.int32, device=dev)
    part = torch.zeros(L.zmi_attention_partial_floats(R, H, Hkv, hd, smax - 1), device=dev)
    cnt = torch.zeros(R * Hkv, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def go():
        _lib.check(L.zmi_attention(q.data_ptr(), H * hd, kc.data_ptr(), vc.data_ptr(), None, rp.data_ptr(), R, H,
                                   Hkv, hd, smax, smax - 1, out.data_ptr(), H * hd, part.data_ptr(), cnt.data_ptr(), s))
    return timed(go)


def empty_kernel():
    x = torch.zeros(1, device=dev)
    return timed(lambda: x.add_(1.0))


def gemv(N, K=2048, M=2, ln=True, epi=_lib.EPI_STORE):
    """ln: False (plain), True (two-pass LayerNorm prologue) or "stats" (partials prologue)."""
    W = torch.randn(N * K, device=dev).to(torch.bfloat16)
    X = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, N, device=dev).to(torch.bfloat16)
    lw, lb = torch.ones(K, device=dev).to(torch.bfloat16), torch.zeros(K, device=dev).to(torch.bfloat16)
    a = _lib.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
    if ln:
        a.ln_w, a.ln_b, a.eps = lw.data_ptr(), lb.data_ptr(), 1e-5
    a.out, a.ldo, a.n_valid = out.data_ptr(), N, N
    s = torch.cuda.current_stream().cuda_stream
    return timed(lambda: _lib.check(L.zmi_gemv_launch(ctypes.byref(a), epi, s)))


if __name__ == "__main__":
    print(json.dumps(dict(probe="torch_add_1elem", us=round(empty_kernel(), 2))), flush=True)
    for R, pos in ((2, 0), (2, 63), (2, 64), (2, 300), (2, 600), (2, 1000), (32, 600)):
        print(json.dumps(dict(probe="attn", R=R, pos=pos, us=round(attn(R, pos), 2))), flush=True)
    for N in (16, 256, 2048, 3072, 16384):
        for ln in (False, True):
            print(json.dumps(dict(probe="gemv_l2_resident", N=N, ln=ln, us=round(gemv(N, ln=ln), 2))), flush=True)
