"""The bench's C5 share (8 voice-clone utterances of 60 s after a 430-frame prefix) on its own.

    python tools/bench_c5.py [n_new]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5168
    print(json.dumps(bench.time_c5(torch.device("cuda", 0), n_new=n)), flush=True)


if __name__ == "__main__":
    main()
