"""The decode-step sampler launch on its own (bench._sampler_us: a graph of back-to-back launches) for greedy
(one-workgroup-per-slot kernel and per-codebook workgroups) and the reference's default min-p sampling
(one JSON line per case)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.engine import SamplingParams  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    e = m.engine
    cond = bench.cond_tensor(0, e.d, dev)
    for rep in range(2):
        for name, prm, gs in (("greedy", dict(temperature=0.0), True), ("greedy", dict(temperature=0.0), False),
                              ("min_p", dict(temperature=1.0, min_p=0.1), True),
                              ("top_p", dict(temperature=1.0, top_p=0.9), True)):
            e.greedy_sampler = gs
            e.prefill(0, cond, None, bench.N_NEW, SamplingParams(cfg_scale=2.0, **prm))
            e.step(8, slots=1)
            us, kind = bench._sampler_us(e, 4)
            e.check_errors()
            e.release(0)
            print(json.dumps(dict(params=name, kernel=kind, us=round(us, 2))), flush=True)


if __name__ == "__main__":
    main()
