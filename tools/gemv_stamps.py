"""Phase timeline of the decode-step GEMVs from the diagnostic build's in-kernel stamps.

    tools/build_gemv_stamps.sh
    ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_gemv_stamps.so python tools/gemv_stamps.py [--layers 3]

Runs the 1-slot decode plan (26 layers + heads, attention included, no sampler) at position 591
and stamps the GEMVs of the first `--layers` layers. Stamps (s_memrealtime, 10 ns) per workgroup:
0 start, 1 weight loads issued, 2 activations in LDS, 3 LayerNorm done, 4 MFMA chain done (all
weights landed), 5 reduction barrier, 6 epilogue done. Per launch: the first workgroup start, the
median of each stamp after it, the last stamp 6 (us), and the gap from the previous stamped launch.
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
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--pos", type=int, default=591)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=1040, max_prefill=16)
    e = m.engine
    e.attn_block = False  # the unfused plan: QKV and attention as their own launches
    with torch.cuda.stream(e.stream):
        e.row_pos[:2] = args.pos
        e.x.normal_()
    e.stream.synchronize()
    buf = torch.zeros(64 * 4096 * 8, dtype=torch.int64, device=dev)
    plan = e._plan(2)
    names, slot = [], 0
    kinds = ["qkv", "out", "fc1", "fc2"]
    gi = 0
    for kind, item in plan:
        if kind != "gemv":
            continue
        layer = gi // 4
        if layer < args.layers and slot < 64:
            item[0].reserved, item[0].diag = slot, buf.data_ptr()
            names.append(f"L{layer}.{kinds[gi % 4]}")
            slot += 1
        gi += 1
    for _ in range(3):
        with torch.cuda.stream(e.stream):
            for kind, item in plan:
                if kind == "gemv":
                    e._run_gemv(item)
                elif kind == "attn":
                    i, apf = item
                    e._attention(i, e.q, 2, None, e.row_pos, e.smax - 1, e.attn, apf)
                else:
                    item()
        e.stream.synchronize()
    st = buf.view(64, 4096, 8).cpu()
    prev_end = None
    for s, name in enumerate(names):
        blk = st[s]
        live = blk[:, 0] > 0
        b = blk[live].double()
        t0 = b[:, 0].min()
        rel = ((b - t0) / 100.0)  # 100 MHz ticks -> us
        med = [round(float(rel[:, i][b[:, i] > 0].median()), 2) if (b[:, i] > 0).any() else None for i in range(7)]
        end = float(((b[:, 6][b[:, 6] > 0]).max() - t0) / 100.0) if (b[:, 6] > 0).any() else None
        last_start = round(float(rel[:, 0].max()), 2)
        gap = None if prev_end is None else round(float((t0 - prev_end) / 100.0), 2)
        ends = rel[:, 6][b[:, 6] > 0]
        q = torch.quantile(ends, torch.tensor([0.1, 0.5, 0.9, 0.99], dtype=torch.float64)).tolist() if len(ends) else []
        idx = live.nonzero().flatten()
        xcd = [round(float(rel[:, 6][(idx % 8 == x) & (b[:, 6] > 0)].median()), 2) for x in range(8)]
        print(json.dumps(dict(launch=name, blocks=int(live.sum()), gap_from_prev_us=gap, last_block_start=last_start,
                              median_stamps_us=med, last_end_us=round(end, 2) if end is not None else None,
                              end_p10_p50_p90_p99=[round(v, 2) for v in q], end_median_by_block_mod8=xcd)))
        prev_end = t0 + (end or 0) * 100.0


if __name__ == "__main__":
    main()
