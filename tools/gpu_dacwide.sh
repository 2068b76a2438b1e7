#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_generate.py -k "dac" > gpurun_out/dacwide_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dacwide_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/dacwide_tests.log | head; exit $rc; }
timeout -k 10 300 python -u tools/dac_wide_ab.py > gpurun_out/dac_wide_ab.jsonl 2> gpurun_out/dac_wide_ab.err
rc=$?; cat gpurun_out/dac_wide_ab.jsonl; tail -2 gpurun_out/dac_wide_ab.err; exit $rc
