#!/bin/bash
# block-form attention x prefetch role, C5-shaped job (8 slots, 2000 new frames)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/blk2.jsonl
for o in '{"attn_variant": 1, "attn_prefetch_blocks": 128}' '{"attn_variant": 0, "attn_prefetch_blocks": 0}' '{"attn_variant": 0, "attn_prefetch_blocks": 128}' '{"attn_variant": 1, "attn_prefetch_blocks": 0}' '{"attn_variant": 0, "attn_prefetch_blocks": 0}' '{"attn_variant": 1, "attn_prefetch_blocks": 128}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 2000 "$o" >> gpurun_out/blk2.jsonl 2>> gpurun_out/blk2.err || exit 4
done
