"""Decode attention at many rows and long contexts (C5: 16 rows x ~3.2k keys) on its own.

    python tools/attn_bench.py [--rows 16] [--pos 3200] [--layers 26] [--reps 3]

Random q / K / V caches for `layers` layers (each launch reads another layer's cache, so K / V come from
HBM as in the decode step, not from the Infinity Cache), zmi_attention_variant per launch timed with HIP
events over all layers back to back. Prints us per launch, the K / V bytes and GB/s.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

HD, HKV, HQ = 128, 4, 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16)
    ap.add_argument("--pos", type=int, default=3200)
    ap.add_argument("--layers", type=int, default=26)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variant", type=int, default=1)
    ap.add_argument("--xc", type=int, default=None, help="ZMI_OPT_XC_HANDOFF (0: hand-offs through the XCD's L2)")
    ap.add_argument("--smax", type=int, default=0, help="KV capacity (default pos + 72)")
    ap.add_argument("--rezero", action="store_true", help="zero the work buffer before every launch (timing-only "
                    "builds that stop early never re-arm their hand-offs)")
    args = ap.parse_args()
    L = _lib.lib()
    if args.xc is not None:
        _lib.check(L.zmi_set_option(_lib.OPT_XC_HANDOFF, args.xc), "set_option")
    dev = "cuda"
    rows, p = args.rows, args.pos
    smax = args.smax or p + 72
    smax += (-smax) % 8
    kc = [torch.randn(rows, HKV, smax, HD, device=dev).to(torch.bfloat16) for _ in range(args.layers)]
    vt = [torch.randn(rows, HKV, HD, smax, device=dev).to(torch.bfloat16) for _ in range(args.layers)]
    q = torch.randn(rows, HQ * HD, device=dev).to(torch.bfloat16)
    out = torch.zeros_like(q)
    rp = torch.full((rows,), p, dtype=torch.int32, device=dev)
    work = torch.zeros(L.zmi_attention_work_bytes(rows, HQ, HKV, HD, smax - 1), dtype=torch.uint8, device=dev)
    nf = L.zmi_attention_partial_floats(rows, HQ, HKV, HD, smax - 1)
    po = torch.zeros(nf, device=dev)
    plm = torch.zeros(nf // HD * 2, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def launch(i):
        if args.rezero:
            work.zero_()
        _lib.check(L.zmi_attention_variant(q.data_ptr(), HQ * HD, kc[i].data_ptr(), vt[i].data_ptr(), None, rp.data_ptr(),
                                           rows, HQ, HKV, HD, smax, smax - 1, out.data_ptr(), HQ * HD, po.data_ptr(),
                                           plm.data_ptr(), work.data_ptr(), args.variant, s))

    for i in range(args.layers):
        launch(i)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(args.reps):
        st.record()
        for i in range(args.layers):
            launch(i)
        en.record()
        en.synchronize()
        ts.append(st.elapsed_time(en) * 1000.0 / args.layers)
    assert args.rezero or int(work[:4].view(torch.int32).item()) == 0, "a hand-off timed out"
    us = min(ts)
    nbytes = rows * HKV * (p + 1) * HD * 2 * 2
    print(json.dumps(dict(lib=os.environ.get("ZMI_LIB_PATH", "default"), xc=args.xc, rows=rows, pos=p, smax=smax, variant=args.variant, rezero=args.rezero,
                          us=round(us, 2), kv_bytes=nbytes, GBps=round(nbytes / us / 1e3, 1))), flush=True)


if __name__ == "__main__":
    main()
