"""Time the many-row split-K GEMM (zmi_gemv_splitk_ln: fc2 K = 8192 / out_proj K = 2048, + residual + LayerNorm) with
its reduce in the same launch (ZMI_OPT_SPLITK_REDUCE = 1) against the two-launch forms (0, 2), alternating the arms in one
process; weights rotate over 26 copies so they come from HBM as in a decode step.

    python tools/splitk_bench.py [--rows 16] [--k 8192] [--reps 20]
    tools/build_variant.sh splitk_stamps -DZMI_SPLITK_STAMPS   # diagnostic build, then:
    ZMI_LIB_PATH=zonos_vibes_amd/var/libsplitk_stamps.so python tools/splitk_bench.py --stamps

--stamps prints, for one fused launch, each phase stamp (median / max over workgroups, us after the first workgroup
start): GEMM workgroups 0 start, 1 partials issued, 2 partials drained; reduce workgroups 4 start, 5 all arrivals
seen, 6 row reduced, 7 LayerNorm written.
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib as L  # noqa: E402

D = 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--stamps", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = L.lib()
    M, K = args.rows, args.k
    g = torch.Generator(device=dev).manual_seed(1)
    stream = torch.cuda.Stream(dev)
    sp = stream.cuda_stream
    ws = []
    for _ in range(26):
        w = (torch.randn(D, K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
        wp = torch.empty(D * K, dtype=torch.bfloat16, device=dev)
        L.check(lib.zmi_pack_weight(w.data_ptr(), wp.data_ptr(), D, K, D, L.PACK_IDENTITY, sp))
        ws.append(wp)
    h = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    xn = torch.zeros(M, D, dtype=torch.bfloat16, device=dev)
    lw = torch.ones(D, dtype=torch.bfloat16, device=dev)
    lb = torch.zeros(D, dtype=torch.bfloat16, device=dev)
    nf = lib.zmi_gemv_splitk_floats(M, D)
    part = torch.zeros(nf, dtype=torch.float32, device=dev)
    diag = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
    stream.synchronize()

    def launch(i, stamped=False):
        a = L.GemvArgs()
        a.W, a.X, a.M, a.N, a.K, a.ldx = ws[i % 26].data_ptr(), h.data_ptr(), M, D, K, K
        a.out, a.ldo, a.n_valid, a.eps = x.data_ptr(), D, D, 1e-5
        a.diag = diag.data_ptr() if stamped else None
        L.check(lib.zmi_gemv_splitk_ln(ctypes.byref(a), L.EPI_RESIDUAL, part.data_ptr(), nf, lw.data_ptr(),
                                       lb.data_ptr(), 1e-5, xn.data_ptr(), D, sp), "splitk_ln")

    res = {}
    names = {0: "two_launches_256", 1: "in_launch", 2: "two_launches_512"}
    for arm in (1, 0, 2, 1, 0, 2, 1, 0, 2):
        L.check(lib.zmi_set_option(L.OPT_SPLITK_REDUCE, arm))
        with torch.cuda.stream(stream):
            for i in range(26):
                launch(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(26 * args.reps):
                launch(i)
            e1.record(stream)
        stream.synchronize()
        res.setdefault(names[arm], []).append(round(e0.elapsed_time(e1) * 1e3 / (26 * args.reps), 2))
    ew = lib.zmi_gemv_splitk_layout(1)
    err = int(part[ew:ew + 1].view(torch.int32).item())
    print(json.dumps(dict(rows=M, k=K, us_per_op=res, err=err)), flush=True)
    if args.stamps:
        L.check(lib.zmi_set_option(L.OPT_SPLITK_REDUCE, 1))
        with torch.cuda.stream(stream):
            for i in range(26):
                launch(i)
            diag.zero_()
            launch(26, stamped=True)
        stream.synchronize()
        st = diag.view(4096, 8).cpu().double()
        n_gemm = (D // 64) * (8 if K == 8192 else 4)
        t0 = st[: n_gemm + M, 0][st[: n_gemm + M, 0] > 0].min()
        t0 = min(float(t0), float(st[n_gemm: n_gemm + M, 4].min()))
        out = {}
        for role, sl, cols in (("gemm", slice(0, n_gemm), (0, 1, 2)), ("reduce", slice(n_gemm, n_gemm + M), (4, 5, 6, 7))):
            blk = st[sl]
            out[role] = {str(c): [round(float((blk[:, c] - t0).median()) / 100, 2), round(float((blk[:, c] - t0).max()) / 100, 2)]
                         for c in cols}
        print(json.dumps(dict(rows=M, k=K, stamps_median_max_us=out)), flush=True)


if __name__ == "__main__":
    main()
