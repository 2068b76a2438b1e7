"""Prefill A/B, arms alternating in one process (weight placement moves timings between processes):

    python tools/prefill_ab.py hybrid|transformer '[{"splitk_m_rows": 16}, {"splitk_m_rows": 0}]' [reps] [nocheck]

An arm is a dict of engine attributes (set, then the plan rebuilt) plus optional "opt:<N>" library knobs
(zmi_set_option). Each arm times the Lc + 1 = 161-row CFG prefill (322 rows) of the bench's C2 / C4 utterance
(HIP events around engine.prefill on the engine stream) and checks that every arm's prefill logits equal the first
arm's. One JSON line per arm: median / min ms over the repetitions.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.engine import SamplingParams  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    kind = sys.argv[1]
    arms = json.loads(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    check = not (len(sys.argv) > 4 and sys.argv[4] == "nocheck")  # arms whose arithmetic differs: times only
    dev = torch.device("cuda", 0)
    from zonos_vibes_amd.config import zonos_v01_hybrid, zonos_v01_transformer
    cfg = zonos_v01_hybrid() if kind == "hybrid" else zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=bench.LC + 64, max_prefill=bench.LC + 1)
    e = m.engine
    cond = bench.cond_tensor(1, cfg.backbone.d_model, dev)
    sp = SamplingParams(temperature=0.0)
    lib = _lib.lib()
    base = {k: getattr(e, k) for a in arms for k in a if not k.startswith("opt:")}
    opt0 = {int(k[4:]): lib.zmi_get_option(int(k[4:])) for a in arms for k in a if k.startswith("opt:")}
    times = [[] for _ in arms]
    ref = None
    for r in range(reps + 1):
        for i, arm in enumerate(arms):
            for k, v in base.items():
                setattr(e, k, v)
            for k, v in opt0.items():
                lib.zmi_set_option(k, v)
            for k, v in arm.items():
                if k.startswith("opt:"):
                    lib.zmi_set_option(int(k[4:]), int(v))
                else:
                    setattr(e, k, v)
            e._build_plan()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            with torch.cuda.stream(e.stream):
                st.record(e.stream)
                e.prefill(0, cond, None, 32, sp)
                en.record(e.stream)
            en.synchronize()
            lg = e.logits_pre.clone() if hasattr(e, "logits_pre") else e.logits.clone()
            e.release(0)
            if ref is None:
                ref = lg
            if check:
                assert torch.equal(lg, ref), f"arm {arm}: prefill logits differ"
            if r:
                times[i].append(st.elapsed_time(en))
    for arm, t in zip(arms, times):
        print(json.dumps({"kind": kind, "arm": arm, "prefill_rows": 2 * (bench.LC + 1),
                          "ms_median": round(statistics.median(t), 3), "ms_min": round(min(t), 3)}), flush=True)


if __name__ == "__main__":
    main()
