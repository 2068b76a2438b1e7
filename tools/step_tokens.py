"""Decode-step time of the persistent step kernel vs its weight-stream token budget.

    python tools/step_tokens.py [--tokens 2,3,4,6,8,16] [--steps 64]

For each budget: fresh C2 prefill, run to about the mean position, time `steps` graph replays
with HIP events on the engine stream. One JSON line {tokens: us_per_step}.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import LC, N_NEW, cond_tensor  # noqa: E402
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.engine import SamplingParams  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="2,3,4,6,8,16")
    ap.add_argument("--steps", type=int, default=64)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, zero_eos=True, max_seqlen=LC + N_NEW + 9, max_prefill=LC + 1)
    e = m.engine
    assert e.step_args is not None
    cond = cond_tensor(1, cfg.backbone.d_model, dev)
    out = {}
    for t in [int(x) for x in args.tokens.split(",")]:
        e.step_args.tokens = t
        if e._graph is not None:
            _lib.check(e.lib.zmi_graph_destroy(e._graph))
            e._graph = None
        e.prefill(0, cond, None, N_NEW, SamplingParams(temperature=0.0))
        e.step(N_NEW // 2 - args.steps // 2)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(e.stream)
        e.step(args.steps)
        s1.record(e.stream)
        s1.synchronize()
        e.check_step()
        out[t] = round(s0.elapsed_time(s1) * 1000 / args.steps, 1)
        e.release(0)
        print(t, out[t], flush=True)
    print(json.dumps({"us_per_step_by_tokens": out}))


if __name__ == "__main__":
    main()
