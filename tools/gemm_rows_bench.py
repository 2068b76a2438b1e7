"""Many-row GEMV timing per launch form (HIP events), arms alternating in one process:

    python tools/gemm_rows_bench.py [rows,...] [ZMI_OPT_GEMM_ROWS values,...]

For each row count and the Zonos-v0.1 K = 2048 shapes (qkv 3072, out_proj 2048, fc1 16384 SwiGLU-packed, heads
9248): zmi_gemv_launch over 8 weight copies in turn (so weights come from HBM, as in a decode step), each form
checked bit-identical to the first. One JSON line per (shape, rows, option): us per launch, weight GB/s.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

SHAPES = {"qkv": 3072, "out_proj": 2048, "fc1": 16384, "heads": 9248}


def main():
    rows = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,128,322").split(",")]
    opts = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,3").split(",")]
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    K, ncopy, reps = 2048, 8, 20
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N in SHAPES.items():
        Ws = [torch.empty(N * K, dtype=torch.bfloat16, device=dev).uniform_(-0.03, 0.03, generator=g)
              for _ in range(ncopy)]
        for M in rows:
            X = torch.empty(M, K, dtype=torch.bfloat16, device=dev).uniform_(-2, 2, generator=g)
            out = torch.zeros(M, N, dtype=torch.float32, device=dev)
            ref = None
            for o in opts:
                _lib.check(lib.zmi_set_option(_lib.OPT_GEMM_ROWS, o))
                args = []
                for W in Ws:
                    a = _lib.GemvArgs()
                    a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
                    a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), N, N, 1e-5
                    args.append(a)
                run = lambda: [_lib.check(lib.zmi_gemv_launch(ctypes.byref(a), _lib.EPI_F32, sp)) for a in args]  # noqa
                with torch.cuda.stream(s):
                    run()
                    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    st.record(s)
                    for _ in range(reps):
                        run()
                    en.record(s)
                en.synchronize()
                us = st.elapsed_time(en) * 1e3 / (reps * ncopy)
                got = out.clone()
                if ref is None:
                    ref = got
                print(json.dumps({"shape": name, "N": N, "rows": M, "opt_gemm_rows": o, "us": round(us, 2),
                                  "weight_GBps": round(N * K * 2 / us / 1e3, 1), "bit_identical": bool(torch.equal(got, ref))}),
                      flush=True)
    _lib.check(lib.zmi_set_option(_lib.OPT_GEMM_ROWS, 1))


if __name__ == "__main__":
    main()
