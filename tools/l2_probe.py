"""Does a buffer read by one kernel stay in the XCDs' L2 for the next kernel, or only in the Infinity Cache?

    python tools/l2_probe.py

A 24 MB bf16 buffer (under the 8 x 4 MiB of L2) is summed by torch's reduction kernel (same grid every launch, so
block b reads the same lines each time): "cold" after a 2 GiB sweep of another buffer, "same" right after summing the
same view, "shifted" right after summing a view offset by 1 MiB (the same lines, read by other blocks: other XCDs for
most of them, so they come from the Infinity Cache, not the reading XCD's L2). HIP events, median of 20.
"""
import json

import torch


def main():
    dev = torch.device("cuda", 0)
    n = 12 * 2 ** 20  # 24 MB of bf16
    off = 2 ** 19     # 1 MiB
    buf = torch.randn(n + off, device=dev).to(torch.bfloat16)
    big = torch.empty(2 ** 30, dtype=torch.bfloat16, device=dev)
    a, b = buf[:n], buf[off:off + n]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(view):
        st.record()
        view.sum()
        en.record()
        en.synchronize()
        return st.elapsed_time(en) * 1000.0

    res = {"cold": [], "same": [], "shifted": []}
    for _ in range(20):
        big.add_(1)
        torch.cuda.synchronize()
        res["cold"].append(timed(a))
        res["same"].append(timed(a))
        big.add_(1)
        b.sum()
        torch.cuda.synchronize()
        res["shifted"].append(timed(a))
    out = {k: round(sorted(v)[len(v) // 2], 2) for k, v in res.items()}
    out["MB"] = n * 2 / 1e6
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
