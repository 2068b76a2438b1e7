"""Phase timeline of the block-form attention (variant 5) from the diagnostic build's in-kernel stamps.

    SRC=zmi_attn tools/build_ab.sh attnstamps -DZMI_ATTN_STAMPS
    ZMI_LIB_PATH=zonos_vibes_amd/ab/libattnstamps.so python tools/attn_blk_stamps.py [--rows 16] [--pos 2600]

Stamps (s_memrealtime, 10 ns) per workgroup: 0 start, 1 q in LDS, 2 scores, 3 block maxima exchanged, 4 P,
5 P.V done (V landed), 6 partial out, 7 end (the unit's last arriver: merge done). One launch over a fresh
layer's cache (K / V from HBM) after warm-up launches on other layers; per block index j: the median of each
stamp after the launch's first workgroup start, and the last end.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

HD, HKV, HQ, CH, BLK = 128, 4, 16, 128, 512


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16)
    ap.add_argument("--pos", type=int, default=2600)
    ap.add_argument("--layers", type=int, default=6)
    args = ap.parse_args()
    L = _lib.lib()
    rows, p = args.rows, args.pos
    smax = p + 72
    smax += (-smax) % 8
    kc = [torch.randn(rows, HKV, smax, HD, device="cuda").to(torch.bfloat16) for _ in range(args.layers)]
    vt = [torch.randn(rows, HKV, HD, smax, device="cuda").to(torch.bfloat16) for _ in range(args.layers)]
    q = torch.randn(rows, HQ * HD, device="cuda").to(torch.bfloat16)
    out = torch.zeros_like(q)
    rp = torch.full((rows,), p, dtype=torch.int32, device="cuda")
    wbytes = L.zmi_attention_work_bytes(rows, HQ, HKV, HD, smax - 1)
    work = torch.zeros(wbytes, dtype=torch.uint8, device="cuda")
    nf = L.zmi_attention_partial_floats(rows, HQ, HKV, HD, smax - 1)
    po, plm = torch.zeros(nf, device="cuda"), torch.zeros(nf // HD * 2, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    units, nch, g = rows * HKV, (smax - 1) // CH + 1, HQ // HKV
    r256 = lambda x: (x + 255) // 256 * 256  # noqa: E731
    st_off = 256 + r256(units * 4) + r256(units * nch * g * 8)
    nbmax = (nch + 3) // 4
    n_att = units * nbmax
    for i in range(args.layers):
        _lib.check(L.zmi_attention_variant(q.data_ptr(), HQ * HD, kc[i].data_ptr(), vt[i].data_ptr(), None,
                                           rp.data_ptr(), rows, HQ, HKV, HD, smax, smax - 1, out.data_ptr(), HQ * HD,
                                           po.data_ptr(), plm.data_ptr(), work.data_ptr(), 5, s))
    torch.cuda.synchronize()
    assert int(work[:4].view(torch.int32).item()) == 0, "a hand-off timed out"
    stamps = work[st_off:st_off + n_att * 64].view(torch.int64).view(n_att, 8).cpu().double()
    live = stamps[:, 0] > 0
    t0 = stamps[live][:, 0].min()
    rel = (stamps - t0) / 100.0
    nb = p // BLK + 1
    res = dict(rows=rows, pos=p, blocks_per_unit=nb, workgroups=int(live.sum()),
               launch_last_end=round(float(rel[live][:, 7].max()), 2))
    for j in range(nb):
        sel = live.clone()
        sel[:] = False
        sel[j * units:(j + 1) * units] = True
        sel &= live
        r = rel[sel]
        res[f"block{j}"] = [round(float(r[:, i].median()), 2) for i in range(8)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
