"""Micro-benchmark of the decode GEMV shapes (M = 2 rows) over launch variants, HIP-event timed.

Weights are rotated over distinct buffers (> 400 MiB in total) so each launch streams from HBM,
as in the decode step. Prints one JSON line per (shape, variant). A torch read-reduction of
the same bytes is timed as the streaming reference of this access volume.
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
SHAPES = {  # name: (N, K, epi, ln)
    "qkv": (3072, 2048, _lib.EPI_STORE, True),
    "out": (2048, 2048, _lib.EPI_RESIDUAL, False),
    "fc1": (16384, 2048, _lib.EPI_SWIGLU, True),
    "fc1_plain": (16384, 2048, _lib.EPI_STORE, False),
    "fc2": (2048, 8192, _lib.EPI_RESIDUAL, False),
    "heads": (9248, 2048, _lib.EPI_STORE, True),
}
VARIANTS = [(1, 0), (1, 1), (1, 2), (2, 0), (2, 1), (4, 0), (4, 1), (8, 1), (16, 1)]  # (ksplit, nchunk; 0 = library choice)


def timed(fn, reps):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) * 1e3 / reps


def run(name, M=2, reps=20):
    N, K, epi, ln = SHAPES[name]
    wbytes = N * K * 2
    copies = max(2, (400 << 20) // wbytes + 1)
    Ws = [torch.randn(N * K, device=dev).to(torch.bfloat16) for _ in range(copies)]
    X = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, max(N, K), device=dev).to(torch.bfloat16)
    lw, lb = torch.ones(K, device=dev).to(torch.bfloat16), torch.zeros(K, device=dev).to(torch.bfloat16)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    acc = torch.zeros((), device=dev)

    def ref():
        for W in Ws:
            acc.add_(W.view(torch.int16).sum(dtype=torch.int32).float())
    us_ref = timed(ref, 3) / len(Ws)
    print(json.dumps(dict(shape=name, variant="torch_int_sum_read", us=round(us_ref, 2),
                          GBps=round(wbytes / us_ref / 1e3, 1))), flush=True)
    for ks, nch in VARIANTS:
        per_wave = (K // 32) // (4 * ks) if (K // 32) % (4 * ks) == 0 else 0
        if not per_wave or (nch and (per_wave % nch or per_wave // nch not in (2, 4, 8, 16))):
            continue
        slab = torch.zeros(max(L.zmi_gemv_slab_floats(M, N, K, ks), 1), device=dev)
        args = []
        for W in Ws:
            a = _lib.GemvArgs()
            a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
            a.ksplit, a.nchunk = ks, nch
            if ln:
                a.ln_w, a.ln_b, a.eps = lw.data_ptr(), lb.data_ptr(), 1e-5
            a.out, a.ldo, a.n_valid = out.data_ptr(), (N // 2 if epi == _lib.EPI_SWIGLU else N), N
            a.slab, a.counters = slab.data_ptr(), cnt.data_ptr()
            a.slab_cap, a.counters_cap = slab.numel(), cnt.numel()
            args.append(a)

        def go():
            for a in args:
                _lib.check(L.zmi_gemv_launch(ctypes.byref(a), epi, s))
        us = timed(go, reps) / len(args)
        print(json.dumps(dict(shape=name, ksplit=ks, nchunk=nch, us=round(us, 2), GBps=round(wbytes / us / 1e3, 1))),
              flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(SHAPES):
        run(n)
