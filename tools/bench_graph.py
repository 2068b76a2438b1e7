"""Graph-captured per-launch times (no host launch floor): decode GEMVs vs a pure streaming read.

Each probe captures `copies` launches (weights rotated over > 1 GiB, so reads come from HBM) into
one hipGraph, replays it, and reports device time per launch (HIP events on the capture stream).
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
SHAPES = {"qkv": (3072, 2048, _lib.EPI_STORE, True), "out": (2048, 2048, _lib.EPI_RESIDUAL, False),
          "fc1": (16384, 2048, _lib.EPI_SWIGLU, True), "fc2": (2048, 8192, _lib.EPI_RESIDUAL, False),
          "heads": (9248, 2048, _lib.EPI_LOGITS, True)}


def graph_time(enqueue, n_launch, stream, reps=5):
    sp = stream.cuda_stream
    with torch.cuda.stream(stream):
        enqueue()  # warm (and first-use attributes) outside capture
    stream.synchronize()
    _lib.check(L.zmi_graph_begin(sp))
    with torch.cuda.stream(stream):
        enqueue()
    g = ctypes.c_void_p()
    _lib.check(L.zmi_graph_end(sp, ctypes.byref(g)))
    _lib.check(L.zmi_graph_launch(g, 1, sp))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    _lib.check(L.zmi_graph_launch(g, reps, sp))
    e1.record(stream)
    e1.synchronize()
    L.zmi_graph_destroy(g)
    return e0.elapsed_time(e1) * 1e3 / (reps * n_launch)


def weights(nbytes, total=1200 << 20):
    copies = max(4, total // nbytes + 1)
    Ws = [torch.empty(nbytes // 2, dtype=torch.bfloat16, device=dev) for _ in range(copies)]
    for W in Ws:
        W.uniform_(-0.05, 0.05)
    return Ws


def probe_read(mb, blocks):
    nbytes = int(mb * 1e6) // 1024 * 1024
    Ws = weights(nbytes)
    s = torch.cuda.Stream()

    def enq():
        for W in Ws:
            _lib.check(L.zmi_prefetch(W.data_ptr(), nbytes, blocks, s.cuda_stream))
    us = graph_time(enq, len(Ws), s)
    print(json.dumps(dict(probe="read", MB=mb, blocks=blocks, us=round(us, 2), GBps=round(nbytes / us / 1e3, 1))),
          flush=True)


def probe_gemv(name, M=2, ksplit=0):
    N, K, epi, ln = SHAPES[name]
    Ws = weights(N * K * 2)
    X = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, 9 * 1026 if epi == _lib.EPI_LOGITS else max(N, K), device=dev)
    outb = torch.zeros(M, max(N, K), device=dev).to(torch.bfloat16)
    lw, lb = torch.ones(K, device=dev).to(torch.bfloat16), torch.zeros(K, device=dev).to(torch.bfloat16)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    slab = torch.zeros(max(L.zmi_gemv_slab_floats(M, N, K, ksplit), 1), device=dev)
    s = torch.cuda.Stream()
    args = []
    for W in Ws:
        a = _lib.GemvArgs()
        a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
        a.ksplit = ksplit
        if ln:
            a.ln_w, a.ln_b, a.eps = lw.data_ptr(), lb.data_ptr(), 1e-5
        if epi == _lib.EPI_LOGITS:
            a.out, a.ldo, a.n_valid = out.data_ptr(), 0, 9 * 1026
        else:
            a.out, a.ldo, a.n_valid = outb.data_ptr(), (N // 2 if epi == _lib.EPI_SWIGLU else N), N
        a.slab, a.counters, a.slab_cap, a.counters_cap = slab.data_ptr(), cnt.data_ptr(), slab.numel(), cnt.numel()
        args.append(a)

    def enq():
        for a in args:
            _lib.check(L.zmi_gemv_launch(ctypes.byref(a), epi, s.cuda_stream))
    us = graph_time(enq, len(args), s)
    print(json.dumps(dict(probe="gemv", shape=name, M=M, ksplit=ksplit, us=round(us, 2),
                          GBps=round(N * K * 2 / us / 1e3, 1))), flush=True)
    del Ws


if __name__ == "__main__":
    what = sys.argv[1:] or ["read", "gemv"]
    if "read" in what:
        for mb in (8.4, 12.6, 33.6, 67.1):
            for blocks in (256, 512, 1024, 2048):
                probe_read(mb, blocks)
                torch.cuda.empty_cache()
    if "gemv" in what:
        for name in SHAPES:
            for g in ((0, -1, -2, -4) if SHAPES[name][1] == 2048 else (0,)):
                probe_gemv(name, ksplit=g)
                torch.cuda.empty_cache()
        probe_gemv("fc2", M=16)  # MFMA strip kernel, for comparison
        probe_gemv("out", M=16)
