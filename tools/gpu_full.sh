#!/bin/bash
# full GPU test suite (stop on a fault), then the default bench line
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/full_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/full_tests.log | head; exit $rc; fi
cat gpurun_out/full_parity_long.json gpurun_out/full_trajectory_long.json 2>/dev/null | head -40
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r04c.log 2>&1; echo "bench rc=$?"
grep -v amdgpu.ids gpurun_out/bench_r04c.log | tail -1 | cut -c1-600
