"""Phase timeline of the hybrid (C4) decode step's Mamba2 launches from the diagnostic build's stamps.

    tools/build_gemv_stamps.sh
    ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_gemv_stamps.so python tools/hybrid_stamps.py [--layers 3]

Runs the 1-slot hybrid decode plan (no sampler) at positions 591, 592, ... (the step role's granule tags change
every step) and stamps the first `--layers` Mamba2 layers: the zmi_mamba_block launch (in_proj workgroups: 0
start, 1 weight loads issued, 2 activations in LDS, 3 LayerNorm done, 4 MFMA chain done, 5 reduction, 6 epilogue
done; step workgroups: 0 start, 2 granules received, 3 raw values in LDS, 6 end) and the GRMS out_proj GEMV.
Per launch and role: the first workgroup start of the launch, the median of each stamp after it, the last end.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd.config import zonos_v01_hybrid  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def summarize(name, blk, t0, sel):
    b = blk[sel].double()
    rel = (b - t0) / 100.0  # 100 MHz ticks -> us
    med = [round(float(rel[:, i][b[:, i] > 0].median()), 2) if (b[:, i] > 0).any() else None for i in range(7)]
    ends = rel[:, 6][b[:, 6] > 0]
    q = torch.quantile(ends, torch.tensor([0.1, 0.5, 0.9, 0.99], dtype=torch.float64)).tolist() if len(ends) else []
    return dict(launch=name, blocks=int(sel.sum()), last_block_start=round(float(rel[:, 0].max()), 2),
                median_stamps_us=med, last_end_us=round(float(ends.max()), 2) if len(ends) else None,
                end_p10_p50_p90_p99=[round(v, 2) for v in q])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--pos", type=int, default=591)
    ap.add_argument("--ig", type=int, default=2, help="column groups per in_proj workgroup the library was built with")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_hybrid(), dev, seed=0, zero_eos=True, max_seqlen=args.pos + 16, max_prefill=16)
    e = m.engine
    with torch.cuda.stream(e.stream):
        e.x.normal_()
    e.stream.synchronize()
    buf = torch.zeros(64 * 4096 * 8, dtype=torch.int64, device=dev)
    plan = e._plan(2)
    names, slot, layer = [], 0, 0
    n_in = None
    for kind, item in plan:
        if kind == "call" and hasattr(item, "args"):
            ia, _ = item.args
            if layer < args.layers:
                ia.reserved, ia.diag = slot, buf.data_ptr()
                names.append((f"L{layer}.mamba_block", True))
                slot += 1
                n_in = ((ia.N // (8 * args.ig)) + 7) // 8 * 8
            pending_out = layer < args.layers
            layer += 1
        elif kind == "gemv" and item[0].pro in (3, 4) and pending_out:  # the GRMS out_proj after a stamped block
            item[0].reserved, item[0].diag = slot, buf.data_ptr()
            names.append((f"L{layer - 1}.out_proj_grms", False))
            slot += 1
            pending_out = False
    for it in range(4):
        with torch.cuda.stream(e.stream):
            e.row_pos[:2] = args.pos + it
            e.row_kv[:2] = torch.arange(2, device=dev, dtype=e.row_kv.dtype)
            for kind, item in plan:
                if kind == "gemv":
                    e._run_gemv(item)
                elif kind == "attnblk":
                    e._run_attn_block(item)
                elif kind == "attn":
                    i, pf = item if isinstance(item, tuple) else (item, None)
                    e._attention(i, e.q, 2, None, e.row_pos, e.smax - 1, e.attn, pf)
                else:
                    item()
        e.stream.synchronize()
    e.check_errors()
    st = buf.view(64, 4096, 8).cpu()
    for s, (name, is_block) in enumerate(names):
        blk = st[s]
        live = blk[:, 0] > 0
        if not live.any():  # a launch the library does not stamp
            continue
        t0 = blk[live][:, 0].double().min()
        idx = torch.arange(4096)
        if is_block:
            print(json.dumps(summarize(name + ".in_proj", blk, t0, live & (idx < n_in))))
            print(json.dumps(summarize(name + ".step", blk, t0, live & (idx >= n_in))))
        else:
            print(json.dumps(summarize(name, blk, t0, live)))


if __name__ == "__main__":
    main()
