"""Phase timeline of the attention kernel from the diagnostic build's in-kernel stamps.

    tools/build_attn_variants.sh --stamps   (builds zonos_vibes_amd/var/libzonos_attn_stamps.so)
    ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_attn_stamps.so python tools/attn_stamps.py [pos ...]

Stamps (s_memrealtime, 10 ns ticks) per workgroup: 0 start, 1 scores in LDS, 2 chunk max, 3 after
the max exchange, 4 P in LDS, 5 partial ready, 6 last arriver's ticket, 7 merge done. Prints, per
position, the median time of each stamp after the launch's first workgroup start (us).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

HD, G, HKV, HQ = 128, 4, 4, 16
VARIANT = int(os.environ.get("ATTN_VARIANT", "1"))  # 2: the scores / finish pair (stamps of the finish launch)


def run(pos_list, slots=1, reps=20):
    L = _lib.lib()
    dev = "cuda"
    rows = 2 * slots
    smax = max(pos_list) + 72
    smax += (-smax) % 8
    nrot = int(os.environ.get("ATTN_ROTATE", "1"))  # > 1: rotate over caches larger than the Infinity Cache together
    kcs = [torch.randn(rows, HKV, smax, HD, device=dev).to(torch.bfloat16) for _ in range(nrot)]
    vts = [torch.randn(rows, HKV, HD, smax, device=dev).to(torch.bfloat16) for _ in range(nrot)]
    q = torch.randn(rows, HQ * HD, device=dev).to(torch.bfloat16)
    out = torch.zeros_like(q)
    for p in pos_list:
        rp = torch.full((rows,), p, dtype=torch.int32, device=dev)
        nbytes = L.zmi_attention_work_bytes(rows, HQ, HKV, HD, smax - 1)
        work = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        ch = L.zmi_attention_chunk()
        nch = (smax - 1) // ch + 1
        nblocks = rows * HKV * nch
        st = work[nbytes - nblocks * 64:].view(torch.int64).view(nblocks, 8)
        nf = L.zmi_attention_partial_floats(rows, HQ, HKV, HD, smax - 1)
        po = torch.zeros(nf, device=dev)
        plm = torch.zeros(nf // HD * 2, device=dev)
        rel, per_unit = [], []
        for it in range(reps):
            st.zero_()
            for k in range(nrot):  # back to back: the last launch's stamps are read
                kc, vt = kcs[(it + k) % nrot], vts[(it + k) % nrot]
                _lib.check(L.zmi_attention_variant(q.data_ptr(), HQ * HD, kc.data_ptr(), vt.data_ptr(), None,
                                                   rp.data_ptr(), rows, HQ, HKV, HD, smax, smax - 1, out.data_ptr(),
                                                   HQ * HD, po.data_ptr(), plm.data_ptr(), work.data_ptr(), VARIANT,
                                                   torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            s = st.cpu()
            live = s[:, 0] > 0
            s = s[live]
            t0 = s[:, 0].min()
            rr = torch.where(s > 0, (s - t0).double() / 100.0, torch.full_like(s, float("nan"), dtype=torch.float64))
            rel.append(rr)
            # per unit (= query row x kv head): its last chunk max (2), its last exchange (3), its merge (7)
            ids = live.nonzero().flatten() // nch
            for u in ids.unique().tolist():
                ru = rr[ids == u]
                per_unit.append([float(ru[:, 0].nan_to_num(-1).max()), float(ru[:, 2].nan_to_num(-1).max()),
                                 float(ru[:, 3].nan_to_num(-1).max()), float(ru[:, 7].nan_to_num(-1).max())])
        r = torch.cat(rel)
        med = [round(float(r[:, i][~r[:, i].isnan()].median()), 2) if (~r[:, i].isnan()).any() else None for i in range(8)]
        mx = [round(float(r[:, i][~r[:, i].isnan()].max()), 2) if (~r[:, i].isnan()).any() else None for i in range(8)]

        def quant(f):
            return [round(float(r[:, i][~r[:, i].isnan()].quantile(f)), 2) if (~r[:, i].isnan()).any() else None
                    for i in range(8)]
        pu = torch.tensor(per_unit)
        unit = {k: [round(float(pu[:, i].quantile(f)), 2) for f in (0.1, 0.5, 0.9, 1.0)]
                for i, k in enumerate(["last_start", "last_chunk_max", "last_exchange", "merged"])}
        print(json.dumps(dict(pos=p, rows=rows, workgroups=int(live.sum()), p10_us=quant(0.1), median_us=med, p90_us=quant(0.9),
                              max_us=mx, per_unit_q10_50_90_100=unit)), flush=True)


if __name__ == "__main__":
    run([int(a) for a in sys.argv[1:]] or [300, 591], slots=int(os.environ.get("ATTN_SLOTS", "1")))
