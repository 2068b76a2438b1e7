"""Launch-latency floor of a graph of dependent kernels on this GPU (MI355X), for the decode-step
design: N tiny kernels captured back to back in one graph, replayed; reports us per kernel.

    python tools/launch_floor.py
"""
import json

import torch


def per_kernel_us(fn, n_kernels, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
        g.replay()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record(s)
        for _ in range(reps):
            g.replay()
        en.record(s)
        en.synchronize()
    return st.elapsed_time(en) * 1000 / (reps * n_kernels)


def main():
    dev = torch.device("cuda", 0)
    n = 130
    small = [torch.zeros(256, device=dev) for _ in range(n + 1)]
    print(json.dumps({"case": "chain of 130 add kernels, 1 KiB each (1 workgroup)",
                      "us": round(per_kernel_us(lambda: [small[i + 1].copy_(small[i]) for i in range(n)], n), 2)}))
    mid = [torch.zeros(2 * 2048, dtype=torch.bfloat16, device=dev) for _ in range(n + 1)]
    print(json.dumps({"case": "chain of 130 copies, 8 KiB each",
                      "us": round(per_kernel_us(lambda: [mid[i + 1].copy_(mid[i]) for i in range(n)], n), 2)}))
    for mb in (2, 8, 32, 64):
        big = [torch.zeros(mb * 2 ** 20 // 4, device=dev) for _ in range(3)]
        k = 26
        us = per_kernel_us(lambda: [big[(i + 1) % 3].copy_(big[i % 3]) for i in range(k)], k)
        print(json.dumps({"case": f"chain of {k} copies, {mb} MiB read + {mb} MiB write", "us": round(us, 2),
                          "GBps": round(2 * mb * 2 ** 20 / (us * 1e-6) / 1e9, 1)}))


if __name__ == "__main__":
    main()
