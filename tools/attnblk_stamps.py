"""Phase timeline of the fused QKV + attention launch (zmi_attn_block) from in-kernel stamps.

    tools/build_attnblk_stamps.sh
    ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_attnblk_stamps.so python tools/attnblk_stamps.py [--pos 591]

Synthetic Zonos-v0.1 engine, 1 slot (2 rows) at position `pos`; layer 3's launch is stamped
(s_memrealtime, 10 ns ticks) after the previous layers ran. Projection role: 0 start, 1 weight
loads issued, 2 activations in LDS, 3 LayerNorm, 4 MFMA chain, 5 reduction, 6 epilogue, 7 counted
in (unused). Attention role: 0 start, 1 q / K / V granules received (wave 0), 2 all scores gathered,
3 chunk maxima, 4 P in LDS, 5 P.V done, 6 output stored. Prints per role the median (and
max) of each stamp after the launch's first workgroup start (us).
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
    ap.add_argument("--slices", type=int, default=8)
    ap.add_argument("--form", default="split",
                    help="split / split24 (chunk workgroups), self (self-scoring) or xs (score exchange)")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-oproj", action="store_true", help="out_proj as its own launch (engine.attn_oproj = False)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=max(1040, args.pos + 24),
                        max_prefill=16)
    e = m.engine
    e.attn_block_slices = e.attn_self_slices = args.slices
    e.attn_oproj = not args.no_oproj
    e.attn_forms = tuple(dict.fromkeys([args.form, "split", "split24", "xs"]))  # the probed form first
    with torch.cuda.stream(e.stream):
        e.row_pos[:2] = args.pos
        e.row_kv[:2] = torch.arange(2, dtype=torch.int32, device=dev)
        e.x.normal_()
    e.stream.synchronize()
    plan = e._plan(2, args.form)
    blocks = [it for kd, it in plan if kd == "attnblk"]
    assert blocks, "the fused plan is not in use"
    buf = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
    stamped = 3
    rows = []
    for _ in range(args.reps):
        buf.zero_()
        e.blk_gran.zero_()  # same position every rep: no granule of the previous rep may match
        with torch.cuda.stream(e.stream):
            for i, it in enumerate(blocks):
                a = it[0]
                a.reserved, a.diag = 0, (buf.data_ptr() if i == stamped else None)
                if len(it) > 4 and it[4] is not None:  # the fused out_proj role stamps into the same buffer
                    it[4].reserved, it[4].diag = 0, a.diag
                e._run_attn_block(it)
                a.diag = None
                if len(it) > 4 and it[4] is not None:
                    it[4].diag = None
        e.stream.synchronize()
        rows.append(buf.view(4096, 8).cpu())
    e.check_errors()
    n_qkv = 192
    out = {}
    n_att = 8 * (24 if args.form == "split24" else 8)
    oproj = any(len(it) > 4 and it[4] is not None for it in blocks)
    roles = [("qkv", slice(0, n_qkv)), ("attention", slice(n_qkv, n_qkv + n_att))]
    if oproj:  # out_proj role: 0 start, 1 weights issued, 7 flags seen, 2 rows gathered, 4 chain, 5 sums, 6 epilogue
        roles.append(("out_proj", slice(n_qkv + n_att, n_qkv + n_att + 128)))
    for role, sl in roles:
        meds, maxs = [[] for _ in range(8)], [[] for _ in range(8)]
        if role == "attention":
            for st in rows:
                st[n_qkv: n_qkv + n_att, 7] = 0
        for st in rows:
            live = st[:, 0] > 0
            t0 = st[live, 0].min()
            blk = st[sl]
            blk = blk[blk[:, 0] > 0].double()
            for i in range(8):
                col = blk[:, i][blk[:, i] > 0]
                if len(col):
                    rel = (col - float(t0)) / 100.0
                    meds[i].append(float(rel.median()))
                    maxs[i].append(float(rel.max()))
        out[role] = dict(median_us=[round(sum(v) / len(v), 2) if v else None for v in meds],
                         max_us=[round(sum(v) / len(v), 2) if v else None for v in maxs])
    print(json.dumps(dict(pos=args.pos, slices=args.slices, form=args.form, oproj=oproj, **out)), flush=True)


if __name__ == "__main__":
    main()
