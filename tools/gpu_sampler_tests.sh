#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sampler_greedy.py tests/test_gpu_fsm.py tests/test_gpu_generate.py tests/test_gpu_engine.py > gpurun_out/s_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s_tests.log; [ $rc -eq 0 ] || grep -E "^FAILED|Error" gpurun_out/s_tests.log | head; exit $rc
