#!/bin/bash
# Round-4 profiling pass (GPU box, repo root): rocprofv3 kernel stats of the default bench, of the long-context
# attention at 16 rows x 3200 keys (tools/attn_bench.py) and of a C5-shaped job; the FETCH_SIZE pass on the fc1
# GEMV that the bench's roofline `traffic` reads. Kept files land in gpurun_out/keep/ (copied to profiles/).
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
mkdir -p gpurun_out/keep
K=gpurun_out/keep
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python bench.py --no-cpu-baseline --no-hybrid --no-batch --no-c5 --no-default-cap > $K/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $K/bench_kernel_stats.csv \;
rm -rf gpurun_out/prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python tools/attn_bench.py --rows 16 --pos 3200 > $K/prof_attn16.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $K/attn16x3200_kernel_stats.csv \;
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python tools/bench_c5.py 2000 > $K/prof_c5.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $K/c5_2000_kernel_stats.csv \;
rm -rf gpurun_out/prof
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fc1 -o pmc -- \
  python tools/pmc_driver.py fc1 > $K/pmc_fc1.log 2>&1 || exit $?
python tools/pmc_summary.py "$(find gpurun_out/pmc_fc1 -name "*counter_collection.csv" -print -quit)" \
  "gemv_kernel<2, 4, 8, 16, 1, 3, 1>" 67158016 > $K/pmc_fc1_fetch.json && rm -rf gpurun_out/pmc_fc1
ls -la $K
