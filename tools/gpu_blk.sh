#!/bin/bash
# the block-form attention as the library choice for >= 32 units: full GPU suite, then C5-shaped and C3-sample A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/blk_tests.log 2>&1 || exit 3
: > gpurun_out/blk.jsonl
for o in '{"attn_variant": 1}' '{"attn_variant": 0}' '{"attn_variant": 1}' '{"attn_variant": 0}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 2000 "$o" >> gpurun_out/blk.jsonl 2>> gpurun_out/blk.err || exit 4
done
for o in '{"attn_variant": 1}' '{"attn_variant": 0}'; do
  timeout -k 10 200 python -u tools/bench_batch.py "$o" >> gpurun_out/blk.jsonl 2>> gpurun_out/blk.err || exit 5
done
