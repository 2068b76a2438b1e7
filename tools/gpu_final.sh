#!/bin/bash
# round-4 final GPU pass: smoke(), the whole -m gpu suite, the default bench, and a C3-share kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/keep
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r04e.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python3 tools/bench_c3.py > gpurun_out/keep/prof_c3.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/keep/c3_share_kernel_stats.csv \;
rm -rf gpurun_out/prof
