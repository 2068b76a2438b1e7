"""The bench's C3-shaped batch sample (64 mixed-length utterances through 64 slots) under a profiler.

    rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o bprof -- python tools/bench_batch.py ['{"knob": v}']

An optional JSON argument sets engine attributes first (A/B runs).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    opts = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
    for k, v in opts.items():
        if k.startswith("opt_"):  # library launch knobs: opt_gemm_rows -> zmi_set_option(OPT_GEMM_ROWS)
            _lib.check(m.engine.lib.zmi_set_option(getattr(_lib, "OPT_" + k[4:].upper()), int(v)), k)
        else:
            setattr(m.engine, k, v)
    m.engine._build_plan()
    print(json.dumps(dict(bench.time_batch(m, dev), opts=opts)), flush=True)


if __name__ == "__main__":
    main()
