#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity_full.py > gpurun_out/parity_full.log 2>&1
rc=$?; tail -3 gpurun_out/parity_full.log; [ $rc -eq 0 ] || grep -E "^FAILED|Error|assert" gpurun_out/parity_full.log | head; exit $rc
