"""Where a decode step's time goes inside the persistent step kernel (diagnostic stamps build).

    python -m zonos_vibes_amd.build --stamps
    ZMI_LIB_PATH=zonos_vibes_amd/libzonos_hip_stamps.so ZMI_STEP_STAMPS=1 python tools/step_stamps.py

Runs the C2 utterance to about its mean position, then one decode step with the kernel's
s_memrealtime stamps on; prints per-layer event times (median over workgroups, us from the
kernel's first stamp) and the mean duration between consecutive chain events. One JSON line.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import LC, N_NEW, cond_tensor  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.engine import SamplingParams  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402

EVENTS = [(1, "qkv_staged"), (11, "qkv_in"), (12, "qkv_done"), (4, "att_q"), (5, "att_pub"), (6, "att_merged"),
          (7, "out_in"), (14, "out_done"), (3, "fc1_staged"), (8, "fc1_in"), (13, "fc1_done"), (9, "fc2_in"),
          (10, "fc2_done")]


def main():
    assert os.environ.get("ZMI_STEP_STAMPS") and "stamps" in os.environ.get("ZMI_LIB_PATH", ""), __doc__
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, zero_eos=True, max_seqlen=LC + N_NEW + 9, max_prefill=LC + 1)
    e = m.engine
    assert e.step_args is not None, "step kernel not selected"
    e.prefill(0, cond_tensor(1, cfg.backbone.d_model, dev), None, N_NEW, SamplingParams(temperature=0.0))
    e.step(N_NEW // 2)
    e.stream.synchronize()
    e.step_stamps.zero_()
    torch.cuda.synchronize()
    e.step(1)
    e.stream.synchronize()
    e.check_step()
    nb, L = e.step_cfg["blocks"], e.L
    st = e.step_stamps[: nb * (L + 1) * 16].view(nb, L + 1, 16).cpu().numpy().astype(np.float64)
    t0 = st[st > 0].min()
    us = np.where(st > 0, (st - t0) / 100.0, np.nan)  # 100 MHz ticks -> us
    med = np.nanmedian(us, axis=0)                      # [L+1][16]
    mx = np.nanmax(us, axis=0)
    per_layer = {name: [round(float(med[l, k]), 2) for l in range(L)] for k, name in EVENTS}
    per_layer_max = {name: [round(float(mx[l, k]), 2) for l in range(L)] for k, name in EVENTS}
    seq = [k for k, _ in EVENTS]
    gaps = {}
    for (k0, n0), (k1, n1) in zip(EVENTS, EVENTS[1:]):
        gaps[f"{n0}->{n1}"] = round(float(np.nanmean(med[1:L - 1, k1] - med[1:L - 1, k0])), 2)
    gaps["fc2_done->next qkv_staged"] = round(float(np.nanmean(med[2:L, 1] - med[1:L - 1, 10])), 2)
    layer_us = float(np.nanmean(np.diff(med[1:L, 1])))
    out = {"layer_us_median_chain": round(layer_us, 2), "gaps_us": gaps,
           "heads_staged_us": round(float(med[L, 3]), 2), "kernel_span_us": round(float(np.nanmax(us)), 2),
           "per_layer_median": per_layer, "per_layer_max": per_layer_max}
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/step_stamps.json", "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("layer_us_median_chain", "gaps_us", "heads_staged_us", "kernel_span_us")}))
    rows = trace_report(e)
    json.dump(rows, open("gpurun_out/step_trace.json", "w"))
    for r in sorted(rows, key=lambda r: (r["b"], r["t"][0])):
        if r["b"] == 0:
            print(r)



def trace_report(e, blocks=(0, 1), layers=(10, 11)):
    """Per-wave task timeline of workgroups `blocks` (stamps build): for each task of `layers`, the
    microseconds spent getting its weights, waiting for its input, computing, and finishing."""
    nb, L = e.step_cfg["blocks"], e.L
    base = nb * (L + 1) * 16
    tr = e.step_stamps[base:].view(8, 16, 128, 8).cpu().numpy()
    t0 = tr[..., 0][tr[..., 0] > 0].min()
    names = {0: "qkv", 1: "att", 2: "out", 3: "fc1", 4: "fc2", 5: "heads", 7: "stage"}
    rows = []
    for b in blocks:
        for w in range(16):
            for q in range(128):
                r = tr[b, w, q]
                if r[0] == 0 or int(r[6]) not in layers:
                    continue
                kind = int(r[7]) & 0xff
                ts = [(x - t0) / 100.0 if x > 0 else None for x in r[:6]]
                rows.append(dict(b=b, w=w, seq=q, l=int(r[6]), kind=names.get(kind, kind), grp=(int(r[7]) >> 8) & 0xffff,
                                 t=[None if x is None else round(x, 2) for x in ts]))
    return rows


if __name__ == "__main__":
    main()
