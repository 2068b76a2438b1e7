#!/bin/bash
# prefetch role in the separate chunked attention launch (> 8 rows): parity of the many-slot paths, then
# C5-shaped (8 slots, 2000 new frames) and C3-sample A/B of its knobs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_splitk.py \
  tests/test_gpu_kernels.py -k "attention or batch or slots" > gpurun_out/apf_tests.log 2>&1 || exit 3
: > gpurun_out/apf.jsonl
for o in '{"attn_prefetch_blocks": 0}' '{"attn_prefetch_blocks": 256}' '{"attn_prefetch_blocks": 256, "attn_prefetch_fc1_mb": 16}' '{"attn_prefetch_blocks": 128}' '{"attn_prefetch_blocks": 0}' '{"attn_prefetch_blocks": 256}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 2000 "$o" >> gpurun_out/apf.jsonl 2>> gpurun_out/apf.err || exit 4
done
for o in '{"attn_prefetch_blocks": 0}' '{"attn_prefetch_blocks": 256}' '{"attn_prefetch_blocks": 0}' '{"attn_prefetch_blocks": 256}'; do
  timeout -k 10 200 python -u tools/bench_batch.py "$o" >> gpurun_out/apf.jsonl 2>> gpurun_out/apf.err || exit 5
done
