#!/bin/bash
# block form, q by LDS-DMA: kernel parity, then the engine-shape timing (16 rows, KV capacity 5784)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k attention > gpurun_out/blk6_tests.log 2>&1 || exit 3
: > gpurun_out/blk6.jsonl
for p in 1000 1600 2600 3200 5000; do
  timeout -k 10 120 python tools/attn_bench.py --rows 16 --pos $p --smax 5784 --variant 0 >> gpurun_out/blk6.jsonl 2>> gpurun_out/blk6.err || exit 4
done
timeout -k 10 120 python tools/attn_bench.py --rows 8 --pos 3200 --smax 5784 --variant 0 >> gpurun_out/blk6.jsonl 2>> gpurun_out/blk6.err || exit 4
timeout -k 10 200 python -u tools/bench_c5.py 2000 >> gpurun_out/blk6.jsonl 2>> gpurun_out/blk6.err || exit 5
