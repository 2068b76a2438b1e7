#!/bin/bash
# block form with block-major order: kernel parity, engine-shape timing, then the C5-shaped job A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k attention > gpurun_out/blk4_tests.log 2>&1 || exit 3
bash tools/gpu_blk3.sh || exit 4
: > gpurun_out/blk2.jsonl
for o in '{"attn_variant": 1}' '{"attn_variant": 0}' '{"attn_variant": 1}' '{"attn_variant": 0}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 2000 "$o" >> gpurun_out/blk2.jsonl 2>> gpurun_out/blk2.err || exit 5
done
