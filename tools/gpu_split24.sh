#!/bin/bash
# 24-chunk split form: fused-block parity (incl. the wide form), long-position parity, then the 30 s batch-1
# line with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_attnblk.py \
  tests/test_gpu_parity_long.py > gpurun_out/s24_tests.log 2>&1 || exit 3
: > gpurun_out/s24.jsonl
for o in '{}' '{"attn_forms": ["split", "xs"]}' '{"attn_forms": ["split", "split24"]}'; do
  timeout -k 10 200 python -u tools/bench_long.py "$o" >> gpurun_out/s24.jsonl 2>> gpurun_out/s24.err || exit 4
done
