"""How fast do the decode GEMVs run when their weights are already in the Infinity Cache (MALL)?

    python tools/mall_probe.py

Synthetic Zonos-v0.1 engine, 1 slot (M = 2 rows). For each GEMV kind: "cold" = the 26 layers'
instances back to back (3.2 GB of weights rotate through, so each launch streams from HBM);
"warm" = layer 0's instance 26 times back to back (its weights stay in L2 / MALL after the first).
HIP events on the engine stream; one JSON line per kind.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=700, max_prefill=16)
    e = m.engine
    e.attn_block = False  # the unfused plan: QKV and attention as their own launches
    rows = 2
    with torch.cuda.stream(e.stream):
        e.row_pos[:rows] = 591
        e.x.normal_()
    e.stream.synchronize()
    plan = e._plan(rows)
    gem = [it for kd, it in plan if kd == "gemv"]
    L = e.L
    kinds = {"qkv": gem[0:4 * L:4], "out_proj": gem[1:4 * L:4], "fc1": gem[2:4 * L:4], "fc2": gem[3:4 * L:4]}
    wbytes = {"qkv": 3072 * 2048 * 2, "out_proj": 2048 * 2048 * 2, "fc1": 16384 * 2048 * 2, "fc2": 2048 * 8192 * 2}
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(items, reps=5):
        with torch.cuda.stream(e.stream):
            for it in items:
                e._run_gemv(it)
            st.record(e.stream)
            for _ in range(reps):
                for it in items:
                    e._run_gemv(it)
            en.record(e.stream)
        en.synchronize()
        return st.elapsed_time(en) * 1000.0 / (reps * len(items))

    for k, items in kinds.items():
        cold = timed(items)
        warm = timed([items[0]] * L)
        print(json.dumps(dict(kind=k, MB=round(wbytes[k] / 1e6, 1), cold_us=round(cold, 2), warm_us=round(warm, 2),
                              cold_GBps=round(wbytes[k] / cold / 1e3, 0), warm_GBps=round(wbytes[k] / warm / 1e3, 0))),
              flush=True)


if __name__ == "__main__":
    main()
