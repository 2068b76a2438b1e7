"""C4 (Zonos-v0.1-hybrid) decode under a profiler: one utterance of N frames after a warm-up.

    rocprofv3 --kernel-trace --stats -d gpurun_out/hyb -o hyb -- python tools/bench_hybrid.py 300
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    print(json.dumps(bench.time_hybrid(torch.device("cuda", 0), n)), flush=True)


if __name__ == "__main__":
    main()
