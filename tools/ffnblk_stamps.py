"""Phase timeline of the fused out_proj + fc1 launch (zmi_ffn_block) from in-kernel stamps.

    tools/build_ffnblk_stamps.sh
    ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_ffnblk_stamps.so python tools/ffnblk_stamps.py [--pos 591]

Synthetic Zonos-v0.1 engine, 1 slot (2 rows) at position `pos`; the decode plan runs up to layer 3's
ffn launch, which is stamped (s_memrealtime, 10 ns) with its granules zeroed first. Stamps of thread 0
per workgroup: 0 start, 1 out_proj operands landed (barrier), 2 out_proj epilogue + granules stored,
3 new residual rows received, 4 barrier after the hand-off, 5 LayerNorm done, 6 fc1 MFMA chains done,
7 SwiGLU epilogue done. Prints the median and max of each stamp after the first workgroup start (us).
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
    with torch.cuda.stream(e.stream):
        e.row_pos[:2] = args.pos
        e.row_kv[:2] = torch.arange(2, dtype=torch.int32, device=dev)
        e.x.normal_()
    e.pos_hi[0] = args.pos
    e.stream.synchronize()
    plan = e._plan(2, e._segments(1, 1)[0][1])
    buf = torch.zeros(256 * 8, dtype=torch.int64, device=dev)
    stamped, rows = 3, []
    for _ in range(args.reps):
        buf.zero_()
        e.ffn_gran.zero_()
        e.blk_gran.zero_()
        with torch.cuda.stream(e.stream):
            for kind, it in plan:
                if kind == "ffnblk":
                    o, f, i = it
                    f.diag = buf.data_ptr() if i == stamped else None
                    e._run_ffn_block(it)
                    f.diag = None
                    if i == stamped:
                        break
                elif kind == "attnblk":
                    e._run_attn_block(it)
                elif kind == "gemv":
                    e._run_gemv(it)
        e.stream.synchronize()
        rows.append(buf.view(256, 8).cpu())
    e.check_errors()
    meds, maxs = [[] for _ in range(8)], [[] for _ in range(8)]
    for st in rows:
        t0 = st[:, 0].min()
        for i in range(8):
            col = (st[:, i] - t0).double() / 100.0
            meds[i].append(float(col.median()))
            maxs[i].append(float(col.max()))
    print(json.dumps(dict(pos=args.pos, median_us=[round(sum(v) / len(v), 2) for v in meds],
                          max_us=[round(sum(v) / len(v), 2) for v in maxs])), flush=True)


if __name__ == "__main__":
    main()
