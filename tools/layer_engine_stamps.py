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

NAMES = ["start", "attention", "attn_rows", "oproj_epi", "x1_rows", "fc1_epi", "h_seg", "combine", "x2_rows", "next_epi"]


def main():
    layer = int(sys.argv[1]) if len(sys.argv) > 1 else 13
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    cond = bench.cond_tensor(1, cfg.backbone.d_model, dev)
    e = m.engine
    res = {}
    for use in (True, False):
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
    diag = torch.zeros(256 * 32, dtype=torch.int64, device=dev)
    plan = e._plan(2, "engine")
    item = plan[1 + layer][1]
    item.diag = diag.data_ptr()
    for _ in range(3):
        e.enqueue_step(slots=1)
    e.stream.synchronize()
    item.diag = None
    e.check_errors()
    d = diag.view(256, 32)[:, :10].cpu().double()
    t0 = d[:, 0].min()
    ph = {n: [round(float((d[:, i] - t0).median()) / 100, 2), round(float((d[:, i] - t0).max()) / 100, 2)]
          for i, n in enumerate(NAMES)}
    res["stamps_us_median_max"] = ph
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
