"""Phase timeline of the fused attention + out_proj + fc1 launch (zmi_attn_ffn_block) from in-kernel stamps.

    tools/build_attnffn_stamps.sh
    ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_attnffn_stamps.so python tools/attnffn_stamps.py [--pos 591]

Synthetic Zonos-v0.1 engine, 1 slot (2 rows) at position `pos`; the decode plan runs up to layer 3's
attn_ffn launch, which is stamped (s_memrealtime, 10 ns) with its granules zeroed first. Stamps of thread 0
per workgroup: 0 start; 1 loads issued (others) / scores in LDS (attention); 2 maxima exchanged; 3 chunk
partials published; 4 attention output published; 5 attention rows gathered; 6 out_proj epilogue + residual
granules; 7 residual rows gathered; 8 barrier S1; 9 LayerNorm done; 10 fc1 chains done; 11 SwiGLU done.
Prints per class (attention workgroups 0..63 with a live chunk, the others) the median and max of each stamp
after the first workgroup start (us).
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
    ap.add_argument("--pos", type=int, default=591)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=1040, max_prefill=16)
    e = m.engine
    from zonos_vibes_amd import _lib
    depth = int(os.environ.get("ZMI_AF_DEPTH", "-1"))
    if depth >= 0:
        _lib.check(e.lib.zmi_set_option(_lib.OPT_AF_DEPTH, depth), "depth")
    delay = int(os.environ.get("ZMI_AF_DELAY", "-1"))
    if delay >= 0:
        _lib.check(e.lib.zmi_set_option(_lib.OPT_AF_DELAY, delay), "delay")
    with torch.cuda.stream(e.stream):
        e.row_pos[:2] = args.pos
        e.row_kv[:2] = torch.arange(2, dtype=torch.int32, device=dev)
        e.x.normal_()
    e.pos_hi[0] = args.pos
    e.stream.synchronize()
    form = e._segments(1, 1)[0][1]
    plan = e._plan(2, form)
    assert any(k == "attnffn" for k, _ in plan), f"form {form}: no attn_ffn launch in the plan"
    buf = torch.zeros(256 * 16, dtype=torch.int64, device=dev)
    stamped, runs = 3, []
    for _ in range(args.reps):
        buf.zero_()
        e.ffn_gran.zero_()
        e.blk_gran.zero_()
        e.attn_gran.zero_()
        with torch.cuda.stream(e.stream):
            for kind, it in plan:
                if kind == "attnffn":
                    a, o, f, i = it
                    f.diag = buf.data_ptr() if i == stamped else None
                    e._run_attn_ffn(it)
                    f.diag = None
                    if i == stamped:
                        break
                elif kind == "gemv":
                    e._run_gemv(it)
        e.stream.synchronize()
        runs.append(buf.view(256, 16).cpu())
    e.check_errors()
    nc = args.pos // 128 + 1
    att = [b for b in range(64) if ((b >> 3) % 8) < nc]
    oth = list(range(64, 256))
    out = dict(pos=args.pos, depth=int(e.lib.zmi_get_option(_lib.OPT_AF_DEPTH)),
               delay=int(e.lib.zmi_get_option(_lib.OPT_AF_DELAY)))
    for name, blocks in (("attention", att), ("others", oth)):
        med, mx = [], []
        for i in range(12):
            vals_m, vals_x = [], []
            for st in runs:
                t0 = st[:, 0][st[:, 0] > 0].min()
                col = st[blocks, i]
                col = col[col > 0]
                if len(col) == 0:
                    continue
                col = (col - t0).double() / 100.0
                vals_m.append(float(col.median()))
                vals_x.append(float(col.max()))
            med.append(round(sum(vals_m) / len(vals_m), 2) if vals_m else None)
            mx.append(round(sum(vals_x) / len(vals_x), 2) if vals_x else None)
        out[name] = dict(median_us=med, max_us=mx)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
