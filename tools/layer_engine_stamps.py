"""Phase stamps of one zmi_layer_engine launch inside a live C2 decode step (full 26-layer dims, synthetic
weights): s_memrealtime (100 MHz) per block at the service phases, medians and maxima in us from the launch's
first stamp. Also times the step (graph replays, HIP events) with the engine plan and with the launch plan.

    python tools/layer_engine_stamps.py [layer]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402

NAMES = {0: "s0_start", 1: "s0_attention", 2: "s0_attn_rows", 3: "s0_oproj_epi", 4: "s0_x1_rows", 5: "s0_fc1_epi",
         6: "s0_h_seg", 7: "s0_combine", 8: "s0_x2_rows", 9: "s0_next_epi",
         10: "att_scores", 11: "att_scores_sync", 12: "att_mj", 13: "att_pv", 14: "att_merged",
         16: "c0_slot0_ready", 17: "c0_fc1_start", 18: "c0_fc2_start", 19: "c0_next_start",
         20: "c0_fc1_done", 21: "c1_fc1_done", 22: "c2_fc1_done", 23: "c3_fc1_done",
         24: "c0_fc2_done", 25: "c1_fc2_done", 26: "c2_fc2_done", 27: "c3_fc2_done",
         28: "s0_att_done", 29: "s1_att_done", 30: "s2_att_done", 31: "s3_att_done",
         32: "s0_f1epi", 33: "s1_f1epi", 34: "s2_f1epi", 35: "s3_f1epi",
         36: "s0_end", 37: "s1_end", 38: "s2_end", 39: "s3_end",
         40: "ld_issued_k0", 41: "ld_issued_k1", 42: "ld_issued_k4", 43: "ld_issued_k8", 44: "ld_issued_k9",
         45: "ld_issued_k12", 46: "ld_issued_k13", 48: "ld_landed_k0", 49: "ld_landed_k8", 50: "ld_landed_k12"}


def main():
    layer = int(sys.argv[1]) if len(sys.argv) > 1 else 13
    from zonos_vibes_amd import _lib
    if len(sys.argv) > 3:  # loader slots in flight, and while a service wave polls
        _lib.check(_lib.lib().zmi_set_option(_lib.OPT_ENG_FLY, int(sys.argv[2])))
        _lib.check(_lib.lib().zmi_set_option(_lib.OPT_ENG_THIN, int(sys.argv[3])))
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    cond = bench.cond_tensor(1, cfg.backbone.d_model, dev)
    e = m.engine
    res = {}
    for use in (True,) + ((False,) if "--launches" in sys.argv else ()):
        e.layer_engine = use
        e._build_plan()
        bench.time_decode_step(m, cond, steps=16)
        us, pos = bench.time_decode_step(m, cond)
        res["step_us_engine" if use else "step_us_launches"] = round(us, 1)
        res["pos"] = pos
    e.layer_engine = True
    e._build_plan()
    from zonos_vibes_amd.engine import SamplingParams
    e.prefill(0, cond, None, 600, SamplingParams(temperature=0.0))
    e.step(431, slots=1)
    diag = torch.zeros(256 * 64, dtype=torch.int64, device=dev)
    plan = e._plan(2, "engine")
    item = plan[1 + layer][1]
    item.diag = diag.data_ptr()
    for _ in range(3):
        e.enqueue_step(slots=1)
    e.stream.synchronize()
    item.diag = None
    e.check_errors()
    d = diag.view(256, 64).cpu().double()
    t0 = d[:, 0].min()
    ph = {}
    for i, n in NAMES.items():
        col = d[:, i]
        sel = col > 0
        if sel.any():
            v = (col[sel] - t0) / 100
            ph[n] = [round(float(v.median()), 2), round(float(v.max()), 2), int(sel.sum())]
    res["stamps_us_median_max_n"] = ph
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
