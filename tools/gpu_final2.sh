#!/bin/bash
# round-4 closing GPU pass: smoke(), the whole -m gpu suite, the default bench, and rocprofv3 kernel stats of
# the bench's C2 path and of a C5-shaped job on the final code (kept files in gpurun_out/keep/)
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
mkdir -p gpurun_out/keep
K=gpurun_out/keep
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $K/final_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $K/final_tests.log 2>&1 || exit $?
tail -2 $K/final_tests.log
timeout -k 10 900 python -u bench.py > $K/bench_r04f.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python bench.py --no-cpu-baseline --no-hybrid --no-batch --no-c5 --no-default-cap > $K/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $K/bench_kernel_stats.csv \;
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python tools/bench_c5.py 2000 > $K/prof_c5.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $K/c5_2000_kernel_stats.csv \;
rm -rf gpurun_out/prof
ls -la $K
