"""The bench's C3 share (bench.time_c3_sharded: 64 of the 512 C3 utterances on one GPU's 64 slots) on its own.

    python tools/bench_c3.py ['{"attn_variant": 1}']   ("opt:<N>": zmi_set_option(N, value))
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    opts = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
    lcs, n_new = bench.c3_job()
    m._ensure_capacity(64, max(lcs[:64]) + max(n_new[:64]) + 9, max(lcs[:64]) + 1)  # the job's engine, then knobs
    from zonos_vibes_amd import _lib
    for k, v in opts.items():
        if k.startswith("opt:"):  # a library knob (zmi_set_option)
            _lib.lib().zmi_set_option(int(k[4:]), int(v))
        else:
            setattr(m.engine, k, v)
    m.engine._build_plan()
    for rep in range(int(os.environ.get("C3_REPS", "1"))):  # a repeat reuses the decode graphs of the first
        r = bench.time_c3_sharded(m, dev, 0, 1, None)
        r["opts"], r["rep"], r["graphs"] = opts, rep, len(m.engine._graphs)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
