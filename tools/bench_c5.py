"""The bench's C5 share (8 voice-clone utterances of 60 s after a 430-frame prefix) on its own.

    python tools/bench_c5.py [n_new] [JSON engine options, e.g. '{"attn_prefetch_blocks": 128}'] [slots]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5168
    opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
    slots = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    r = bench.time_c5(torch.device("cuda", 0), slots=slots, n_new=n, engine_opts=opts)
    r["engine_opts"] = opts
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
