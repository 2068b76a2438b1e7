#!/bin/bash
# two-launch chunked attention: parity, then timing against the one-launch form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k attention > gpurun_out/two_tests.log 2>&1 || exit 3
: > gpurun_out/two.jsonl
for v in 1 5; do
  for rp in "16 1500" "16 3200" "16 5700" "2 1500" "2 3200" "8 3200" "128 1000"; do
    set -- $rp
    timeout -k 10 120 python tools/attn_bench.py --rows $1 --pos $2 --variant $v >> gpurun_out/two.jsonl 2>> gpurun_out/two.err || exit 4
  done
done
