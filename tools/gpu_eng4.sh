#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layer_engine.py -k "590" > gpurun_out/eng4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/eng4_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for ft in "8 4" "8 8" "8 1"; do
  timeout -k 10 200 python -u tools/layer_engine_stamps.py 13 $ft > gpurun_out/eng4_stamps_${ft// /_}.log 2>&1; echo "stamps $ft rc=$?"
  grep -v amdgpu.ids gpurun_out/eng4_stamps_${ft// /_}.log | tail -1
done
