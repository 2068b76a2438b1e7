"""C4 (Zonos-v0.1-hybrid) decode under a profiler: one utterance of N frames after a warm-up.

    rocprofv3 --kernel-trace --stats -d gpurun_out/hyb -o hyb -- python tools/bench_hybrid.py 300
    python tools/bench_hybrid.py 300 '{"opt_xc_handoff": 1}'
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    from zonos_vibes_amd import _lib
    for k, v in (json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}).items():  # library knobs: {"opt_xc_handoff": 1}
        _lib.check(_lib.lib().zmi_set_option(getattr(_lib, "OPT_" + k[4:].upper()), int(v)), k)
    print(json.dumps(bench.time_hybrid(torch.device("cuda", 0), n)), flush=True)


if __name__ == "__main__":
    main()
