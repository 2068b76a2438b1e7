#!/bin/bash
# last GPU pass of the round on the committed tree: smoke(), the whole -m gpu suite, the default bench
set -o pipefail
mkdir -p gpurun_out/keep
K=gpurun_out/keep
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $K/close_smoke.log 2>&1 || exit $?
tail -1 $K/close_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $K/close_tests.log 2>&1 || exit $?
tail -1 $K/close_tests.log
timeout -k 10 900 python -u bench.py > $K/bench_r04g.log 2>&1 || exit $?
grep -v amdgpu.ids $K/bench_r04g.log | tail -1 | cut -c1-300
