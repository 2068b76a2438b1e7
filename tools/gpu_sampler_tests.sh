#!/bin/bash
# the sampler kernels' GPU tests, then their launch times (tools/sampler_bench.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sampler_greedy.py tests/test_gpu_fsm.py tests/test_gpu_generate.py tests/test_gpu_engine.py \
  tests/test_gpu_kernels.py tests/test_gpu_api.py > gpurun_out/s_tests.log 2>&1
rc=$?; tail -2 gpurun_out/s_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/s_tests.log | head; exit $rc; }
timeout -k 10 300 python -u tools/sampler_bench.py > gpurun_out/sampler_bench.jsonl 2> gpurun_out/sampler_bench.err
rc=$?; cat gpurun_out/sampler_bench.jsonl; exit $rc
