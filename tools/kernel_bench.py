"""Per-kernel decode-step timing at the C2 configuration (Zonos-v0.1 dims) on MI355X.

    python tools/kernel_bench.py [--slots 1] [--pos 591] [--reps 5]

Builds the synthetic engine, fills slot positions to `pos` (KV content is synthetic), then times
each kind of launch of the decode plan separately with HIP events on the engine stream: all 26
layers' instances back to back (so each weight comes from HBM, as in the step), `reps` times.
Prints one JSON line per kernel kind with us/launch, algorithmic bytes and GB/s, then the whole
step (graph replay).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=1)
    ap.add_argument("--pos", type=int, default=591)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--attn-variants", default="0,1,4,8", help="zmi_attention_variant choices to time")
    ap.add_argument("--spread", type=int, default=1, help="zmi_set_option(OPT_GEMV_SPREAD)")
    ap.add_argument("--gemm-rows", default="3", help="zmi_set_option(OPT_GEMM_ROWS) values (0 off, 1 M8, 3 dense pairs) to time the GEMVs under")
    args = ap.parse_args()
    _lib.check(_lib.lib().zmi_set_option(_lib.OPT_GEMV_SPREAD, args.spread))
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=args.pos + 64, max_prefill=16,
                        max_slots=args.slots)
    e = m.engine
    rows = 2 * args.slots
    with torch.cuda.stream(e.stream):
        e.row_pos[:rows] = args.pos
        e.row_kv[:rows] = torch.arange(rows, dtype=torch.int32, device=dev)
        e.x.normal_()
        e.kc.normal_()
        e.vc.normal_()
    e.stream.synchronize()
    e.attn_block = False  # the per-kernel breakdown of the unfused plan first
    plan = e._plan(rows)
    kinds = {"qkv": _lib.EPI_QKV, "swiglu(fc1)": _lib.EPI_SWIGLU, "logits(heads)": _lib.EPI_LOGITS}
    groups = {k: [it for kd, it in plan if kd == "gemv" and it[1] == epi] for k, epi in kinds.items()}
    res = [it for kd, it in plan if kd == "gemv" and it[1] == _lib.EPI_RESIDUAL]
    groups["out_proj"], groups["fc2"] = res[0::2], res[1::2]
    d, F, L = e.d, e.F, e.L
    wbytes = {"qkv": 3072 * d * 2, "out_proj": d * d * 2, "swiglu(fc1)": 2 * F * d * 2, "fc2": d * F * 2,
              "logits(heads)": 9 * 1025 * d * 2}
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, n):
        with torch.cuda.stream(e.stream):
            fn()
            st.record(e.stream)
            for _ in range(args.reps):
                fn()
            en.record(e.stream)
        en.synchronize()
        return st.elapsed_time(en) * 1000.0 / (args.reps * n)

    out = {}
    rows_opts = [int(v) for v in args.gemm_rows.split(",")]
    for ro in rows_opts:
        _lib.check(_lib.lib().zmi_set_option(_lib.OPT_GEMM_ROWS, ro))
        for name, items in groups.items():
            us = timed(lambda: [e._run_gemv(it) for it in items], len(items))
            gbs = wbytes[name] / (us * 1e-6) / 1e9
            key = name if ro == rows_opts[0] else f"{name}_rows{ro}"
            out[key] = dict(us=round(us, 2), weight_bytes=wbytes[name], GBps=round(gbs, 1),
                            hbm_frac=round(gbs / 8000, 3), gemm_rows=ro)
    _lib.check(_lib.lib().zmi_set_option(_lib.OPT_GEMM_ROWS, rows_opts[0]))
    kv = rows * e.Hkv * e.hd * 2 * 2 * (args.pos + 1)
    variants = [int(v) for v in args.attn_variants.split(",")]
    for var in variants:
        e.attn_variant = var
        us = timed(lambda: [e._attention(i, e.q, rows, None, e.row_pos, e.smax - 1, e.attn) for i in range(L)], L)
        key = "attention" if var == variants[0] else f"attention_v{var}"
        out[key] = dict(us=round(us, 2), variant=var, kv_bytes=kv, GBps=round(kv / (us * 1e-6) / 1e9, 1))
    e.attn_variant = variants[0]
    e.check_errors()
    for k, v in out.items():
        print(json.dumps(dict(kernel=k, slots=args.slots, pos=args.pos, spread=args.spread, **v)), flush=True)
    per_layer = sum(out[k]["us"] for k in ("qkv", "attention", "out_proj", "swiglu(fc1)", "fc2"))
    print(json.dumps(dict(kernel="sum_per_layer", us=round(per_layer, 2), step_estimate_us=round(
        per_layer * L + out["logits(heads)"]["us"], 1))), flush=True)


if __name__ == "__main__":
    main()
