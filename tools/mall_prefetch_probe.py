"""Does reading a decode GEMV's weights just before it (a plain streaming read, as a concurrent
prefetcher would) make that GEMV faster? Per kind: the GEMV alone after a 1 GiB flush ("cold"),
and after a flush then a full read of its weights ("prefetched"); single launches, HIP events.

    python tools/mall_prefetch_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=700, max_prefill=16)
    e = m.engine
    e.attn_block = False  # the unfused plan: QKV and attention as their own launches
    with torch.cuda.stream(e.stream):
        e.row_pos[:2] = 591
        e.x.normal_()
    e.stream.synchronize()
    gem = [it for kd, it in e._plan(2) if kd == "gemv"]
    lw = e.w["layers"][5]
    kinds = {"qkv": (gem[20], lw["qkv"]), "out_proj": (gem[21], lw["out"]), "fc1": (gem[22], lw["fc1"]),
             "fc2": (gem[23], lw["fc2"])}
    flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k, (item, w) in kinds.items():
        res = {}
        for mode in ("cold", "prefetched", "cold", "prefetched"):
            with torch.cuda.stream(e.stream):
                flush.add_(1.0)
                if mode == "prefetched":
                    w.view(torch.int32).sum()
                st.record(e.stream)
                e._run_gemv(item)
                en.record(e.stream)
            en.synchronize()
            res.setdefault(mode, []).append(round(st.elapsed_time(en) * 1000, 2))
        print(json.dumps(dict(kind=k, MB=round(w.numel() * w.element_size() / 1e6, 1), **res)), flush=True)


if __name__ == "__main__":
    main()
