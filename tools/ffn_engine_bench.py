"""Time the persistent FFN engine (zmi_ffn_engine) against out_proj + fc1 + fc2 as three GEMV launches, at the
Zonos-v0.1 dims, 2 rows, 26 layers of distinct weights (each launch's weights come from HBM), HIP events
around 26-layer passes. Also dumps the engine's phase stamps of one pass.

    python tools/ffn_engine_bench.py [passes]
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_engine import D, F, _engine, _gemv, _weights  # noqa: E402
from tests.test_gpu_kernels import DEV, _lib, rnd  # noqa: E402


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    L = _lib()
    NL, M = 26, 2
    layers = [_weights(1000 + 10 * i) for i in range(NL)]
    attn = rnd(M, D, scale=1.0, seed=5)
    x0 = rnd(M, D, scale=2.0, seed=6)
    h = torch.zeros(M, F, dtype=torch.bfloat16, device=DEV)
    gran = torch.zeros(NL, L.diag().zmi_ffn_engine_gran_words(M), dtype=torch.int64, device=DEV)
    err = torch.zeros(4, dtype=torch.int32, device=DEV)
    pos = [10]

    def launches():
        x = x0.clone()
        for Po, Pf, P2, ln in layers:
            _gemv(L, Po, attn, M, D, D, x, D, L.EPI_RESIDUAL)
            _gemv(L, Pf, x, M, 2 * F, D, h, F, L.EPI_SWIGLU, ln=ln)
            _gemv(L, P2, h, M, D, F, x, D, L.EPI_RESIDUAL)
        return x

    def engine(diag=None):
        x = x0.clone()
        pos[0] += 1
        rp = torch.tensor([pos[0]] * M, dtype=torch.int32, device=DEV)
        for i, (Po, Pf, P2, ln) in enumerate(layers):
            _engine(L, Po, Pf, P2, ln, attn, x, None, rp, gran[i], err, diag=diag if i == NL // 2 else None)
        return x

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(passes):
            out = fn()
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) * 1000 / passes / NL, out

    starts = [int(v) for v in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["1"])]
    for st in starts:
        L.check(L.lib().zmi_set_option(L.OPT_ENG_START, st))
        us, _ = timeit(engine)
        print(json.dumps(dict(start=st, us_per_layer_engine=round(us, 2))), flush=True)
    us_l, xl = timeit(launches)
    us_e, xe = timeit(engine)
    us_l2, _ = timeit(launches)
    us_e2, _ = timeit(engine)
    diag = torch.zeros(256 * 16, dtype=torch.int64, device=DEV)
    engine(diag)
    torch.cuda.synchronize()
    d = diag.view(256, 16).cpu().double()
    t0 = d[:, 0].min()
    names = {0: "start", 1: "oproj_epi", 2: "x_gathered", 3: "ln2", 4: "fc1_epi", 5: "h_gathered", 6: "combined",
             7: "c0_slot0_landed", 8: "c0_oproj", 9: "c0_fc1", 10: "c0_fc2"}
    ph = {n: [round(float((d[:, i] - t0).median()) / 100, 2), round(float((d[:, i] - t0).max()) / 100, 2)]
          for i, n in names.items()}
    bytes_layer = (D * D + 2 * F * D + D * F) * 2
    print(json.dumps(dict(us_per_layer_launches=[round(us_l, 2), round(us_l2, 2)],
                          us_per_layer_engine=[round(us_e, 2), round(us_e2, 2)],
                          engine_tbps=round(bytes_layer / (min(us_e, us_e2) * 1e-6) / 1e12, 3),
                          equal=bool(torch.equal(xl, xe)), err=int(err[0].item()),
                          stamps_us_median_max=ph)), flush=True)


if __name__ == "__main__":
    main()
