"""Split-K GEMM timing per knob setting (HIP events over 8 rotating weight copies, so weights come from HBM):

    python tools/splitk_bench.py [rows,...] '[{"17": 1}, {"17": 0}]'

An arm maps zmi_set_option knob numbers to values. Shapes: fc2 (K 8192, residual), out_proj (K 2048, residual), the
hybrid's Mamba2 out_proj (K 4096, store). Every arm's output is checked bit-identical to the first arm's.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

SHAPES = {"fc2": (8192, _lib.EPI_RESIDUAL), "out_proj": (2048, _lib.EPI_RESIDUAL), "mamba_out": (4096, _lib.EPI_STORE)}


def main():
    rows = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16,128,322").split(",")]
    arms = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{"17": 1}, {"17": 0}]
    dev = torch.device("cuda", 0)
    lib = _lib.lib()
    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    N, ncopy, reps = 2048, 8, 20
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (K, epi) in SHAPES.items():
        Ws = [torch.empty(N * K, dtype=torch.bfloat16, device=dev).uniform_(-0.03, 0.03, generator=g) for _ in range(ncopy)]
        for M in rows:
            X = torch.empty(M, K, dtype=torch.bfloat16, device=dev).uniform_(-2, 2, generator=g)
            out = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            nf = int(lib.zmi_gemv_splitk_floats(M, N))
            part = torch.zeros(nf, dtype=torch.float32, device=dev)
            ref = None
            for arm in arms:
                old = {int(k): lib.zmi_get_option(int(k)) for k in arm}
                for k, v in arm.items():
                    lib.zmi_set_option(int(k), int(v))
                args = []
                for W in Ws:
                    a = _lib.GemvArgs()
                    a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
                    a.out, a.ldo, a.n_valid, a.eps = out.data_ptr(), N, N, 1e-5
                    args.append(a)

                def run():
                    for a in args:
                        _lib.check(lib.zmi_gemv_splitk(ctypes.byref(a), epi, part.data_ptr(), nf, sp), "splitk")

                with torch.cuda.stream(s):
                    out.zero_()
                    args[0].W = Ws[0].data_ptr()
                    _lib.check(lib.zmi_gemv_splitk(ctypes.byref(args[0]), epi, part.data_ptr(), nf, sp), "splitk")
                    got = out.clone()
                    run()
                    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    st.record(s)
                    for _ in range(reps):
                        run()
                    en.record(s)
                en.synchronize()
                for k, v in old.items():
                    lib.zmi_set_option(k, v)
                us = st.elapsed_time(en) * 1e3 / (reps * ncopy)
                if ref is None:
                    ref = got
                print(json.dumps({"shape": name, "K": K, "rows": M, "arm": arm, "us_gemm_plus_reduce": round(us, 2),
                                  "bit_identical": bool(torch.equal(got, ref))}), flush=True)


if __name__ == "__main__":
    main()
