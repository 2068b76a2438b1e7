#!/bin/bash
# rocprof summary of the 16 x 3200 attention at the engine's launch shape (library choice), and the prefetch
# role A/B with the block form in the C5-shaped job
set -o pipefail
mkdir -p gpurun_out/keep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python tools/attn_bench.py --rows 16 --pos 3200 --smax 5784 --variant 0 > gpurun_out/keep/prof_attn16e.log 2>&1 || exit 3
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/keep/attn16x3200_engine_kernel_stats.csv \;
rm -rf gpurun_out/prof
: > gpurun_out/blk5.jsonl
for o in '{"attn_prefetch_blocks": 0}' '{"attn_prefetch_blocks": 128}' '{"attn_prefetch_blocks": 256}' '{"attn_prefetch_blocks": 0}' '{"attn_prefetch_blocks": 128}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 2000 "$o" >> gpurun_out/blk5.jsonl 2>> gpurun_out/blk5.err || exit 4
done
