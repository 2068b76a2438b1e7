"""Phase timeline of the many-row GEMVs (gemm_rows_kernel) from the diagnostic build's in-kernel stamps.

    tools/build_gemv_stamps.sh
    ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_gemv_stamps.so python tools/gemm_rows_stamps.py [--slots 64]

Runs the multi-slot decode plan (attention included, fused blocks off) at `--pos` and stamps the GEMVs of
the first `--layers` layers. Stamps (s_memrealtime, 10 ns) per workgroup: 0 start,
2 second tile's start, 3 its chains done, 4 its barrier passed, 5 its epilogue done, 7 end (stamp 1: the first
tile's chains done). Per launch: the median of each stamp after
the first workgroup's start and the last end (us).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--slots", type=int, default=64)
    ap.add_argument("--pos", type=int, default=600)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=args.pos + 64, max_prefill=16,
                        max_slots=args.slots)
    e = m.engine
    e.attn_block = False
    rows = 2 * args.slots
    with torch.cuda.stream(e.stream):
        e.row_pos[:rows] = args.pos
        e.row_kv[:rows] = torch.arange(rows, dtype=torch.int32, device=dev)
        e.x.normal_()
    e.stream.synchronize()
    buf = torch.zeros(64 * 4096 * 8, dtype=torch.int64, device=dev)
    plan = e._plan(rows)
    names, slot, gi = [], 0, 0
    kinds = ["qkv", "out", "fc1", "fc2"]
    for kind, item in plan:
        if kind != "gemv":
            continue
        layer = gi // 4
        name = f"L{layer}.{kinds[gi % 4]}" if layer < e.L else "heads"
        if (layer < args.layers or name == "heads") and slot < 64:
            item[0].reserved, item[0].diag = slot, buf.data_ptr()
            names.append(name)
            slot += 1
        gi += 1
    for _ in range(3):
        with torch.cuda.stream(e.stream):
            for kind, item in plan:
                if kind == "gemv":
                    e._run_gemv(item)
                elif kind == "attn":
                    i, pf = item if isinstance(item, tuple) else (item, None)
                    e._attention(i, e.q, rows, None, e.row_pos, e.smax - 1, e.attn, pf)
        e.stream.synchronize()
    st = buf.view(64, 4096, 8).cpu()
    for s, name in enumerate(names):
        blk = st[s]
        live = blk[:, 0] > 0
        b = blk[live].double()
        t0 = b[:, 0].min()
        rel = (b - t0) / 100.0
        med = [round(float(rel[:, i][b[:, i] > 0].median()), 2) if (b[:, i] > 0).any() else None for i in range(8)]
        end = float(((b[:, 7][b[:, 7] > 0]).max() - t0) / 100.0) if (b[:, 7] > 0).any() else None
        print(json.dumps(dict(launch=name, blocks=int(live.sum()), last_block_start=round(float(rel[:, 0].max()), 2),
                              median_stamps_us=med, last_end_us=None if end is None else round(end, 2))))


if __name__ == "__main__":
    main()
