"""Does an Infinity-Cache (MALL) prefetch make the decode GEMVs faster?

For each decode GEMV shape (M = 2): weights rotated over > 1 GiB so a plain launch streams from
HBM ("cold"); then the same launch right after zmi_prefetch of its weight ("warm", prefetch not
timed); and the prefetch kernel's own read rate. Also a concurrent variant: prefetch of the NEXT
weight on a second stream while the GEMV of this one runs. HIP events; one JSON line per probe.
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
          "fc1": (16384, 2048, _lib.EPI_SWIGLU, True), "fc2": (2048, 8192, _lib.EPI_RESIDUAL, False)}


def ev():
    return torch.cuda.Event(enable_timing=True)


def run(name, M=2, ksplit=0, nchunk=0, blocks=0):
    N, K, epi, ln = SHAPES[name]
    wbytes = N * K * 2
    copies = max(4, (1200 << 20) // wbytes + 1)
    Ws = [torch.empty(N * K, dtype=torch.bfloat16, device=dev) for _ in range(copies)]
    for W in Ws:
        W.uniform_(-1, 1)
    X = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, max(N, K), device=dev).to(torch.bfloat16)
    lw, lb = torch.ones(K, device=dev).to(torch.bfloat16), torch.zeros(K, device=dev).to(torch.bfloat16)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
    slab = torch.zeros(max(L.zmi_gemv_slab_floats(M, N, K, ksplit), 1), device=dev)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    args = []
    for W in Ws:
        a = _lib.GemvArgs()
        a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
        a.ksplit, a.nchunk = ksplit, nchunk
        if ln:
            a.ln_w, a.ln_b, a.eps = lw.data_ptr(), lb.data_ptr(), 1e-5
        a.out, a.ldo, a.n_valid = out.data_ptr(), (N // 2 if epi == _lib.EPI_SWIGLU else N), N
        a.slab, a.counters, a.slab_cap, a.counters_cap = slab.data_ptr(), cnt.data_ptr(), slab.numel(), cnt.numel()
        args.append(a)
    sp1, sp2 = s1.cuda_stream, s2.cuda_stream
    torch.cuda.synchronize()

    def gemv(a, sp):
        _lib.check(L.zmi_gemv_launch(ctypes.byref(a), epi, sp))

    def pf(W, sp):
        _lib.check(L.zmi_prefetch(W.data_ptr(), W.numel() * 2, blocks, sp))

    res = {}
    # cold, back to back
    with torch.cuda.stream(s1):
        for a in args:
            gemv(a, sp1)
        e0, e1 = ev(), ev()
        e0.record(s1)
        for a in args:
            gemv(a, sp1)
        e1.record(s1)
    e1.synchronize()
    res["cold_us"] = e0.elapsed_time(e1) * 1e3 / len(args)
    # prefetch alone
    with torch.cuda.stream(s1):
        e0, e1 = ev(), ev()
        e0.record(s1)
        for W in Ws:
            pf(W, sp1)
        e1.record(s1)
    e1.synchronize()
    res["prefetch_us"] = e0.elapsed_time(e1) * 1e3 / len(Ws)
    res["prefetch_GBps"] = wbytes / res["prefetch_us"] / 1e3
    # warm: prefetch (untimed) then gemv (timed)
    tot = 0.0
    with torch.cuda.stream(s1):
        evs = []
        for W, a in zip(Ws, args):
            pf(W, sp1)
            e0, e1 = ev(), ev()
            e0.record(s1)
            gemv(a, sp1)
            e1.record(s1)
            evs.append((e0, e1))
    torch.cuda.synchronize()
    tot = sum(a.elapsed_time(b) for a, b in evs)
    res["warm_us"] = tot * 1e3 / len(args)
    # pipelined: prefetch(j+1) on s2 overlaps gemv(j) on s1; gemv(j) waits for prefetch(j);
    # prefetch(j+1) waits for gemv(j-1) (bounded look-ahead of one weight)
    e0, e1 = ev(), ev()
    done = [ev() for _ in Ws]
    gdone = [ev() for _ in Ws]
    e0.record(s1)
    s2.wait_stream(s1)
    with torch.cuda.stream(s2):
        pf(Ws[0], sp2)
        done[0].record(s2)
    for j, a in enumerate(args):
        if j + 1 < len(Ws):
            with torch.cuda.stream(s2):
                if j >= 1:
                    s2.wait_event(gdone[j - 1])
                pf(Ws[j + 1], sp2)
                done[j + 1].record(s2)
        with torch.cuda.stream(s1):
            s1.wait_event(done[j])
            gemv(a, sp1)
            gdone[j].record(s1)
    e1.record(s1)
    torch.cuda.synchronize()
    res["pipelined_us"] = e0.elapsed_time(e1) * 1e3 / len(args)
    out_ = dict(shape=name, ksplit=ksplit, nchunk=nchunk, pf_blocks=blocks, MB=round(wbytes / 1e6, 1))
    out_.update({k: round(v, 2) for k, v in res.items()})
    out_["cold_GBps"] = round(wbytes / res["cold_us"] / 1e3, 1)
    out_["warm_GBps"] = round(wbytes / res["warm_us"] / 1e3, 1)
    out_["pipelined_GBps"] = round(wbytes / res["pipelined_us"] / 1e3, 1)
    print(json.dumps(out_), flush=True)
    del Ws
    torch.cuda.empty_cache()


if __name__ == "__main__":
    for n in SHAPES:
        for blocks in (256, 1024):
            run(n, blocks=blocks)
