#!/bin/bash
# block form vs chunked at the engine's launch shape (max_pos = KV capacity 5783, rows below it)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/blk3.jsonl
for v in 1 5; do
  for p in 1000 1600 2600 5000; do
    timeout -k 10 120 python tools/attn_bench.py --rows 16 --pos $p --smax 5784 --variant $v >> gpurun_out/blk3.jsonl 2>> gpurun_out/blk3.err || exit 4
    timeout -k 10 120 python tools/attn_bench.py --rows 16 --pos $p --variant $v >> gpurun_out/blk3.jsonl 2>> gpurun_out/blk3.err || exit 4
  done
done
