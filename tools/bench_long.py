"""The bench's 30 s batch-1 line (bench.time_long_utterance) on its own, optionally with engine attributes.

    python tools/bench_long.py ['{"attn_forms": ["split", "xs"]}']
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    opts = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
    r = bench.time_long_utterance(torch.device("cuda", 0), engine_opts=opts)
    r["engine_opts"] = opts
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
