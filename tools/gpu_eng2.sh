#!/bin/bash
# round-4 engine pass: engine tests (stop on failure), then timings
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_layer_engine.py > gpurun_out/eng2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/eng2_tests.log | head -30
if [ $rc -ne 0 ]; then tail -40 gpurun_out/eng2_tests.log; exit $rc; fi
timeout -k 10 300 python -u tools/layer_engine_stamps.py 13 > gpurun_out/eng2_stamps.log 2>&1; echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/eng2_stamps.log | tail -3
timeout -k 10 200 python -u tools/ffn_engine_bench.py 20 0,1 > gpurun_out/eng2_ffn.log 2>&1; echo "ffn rc=$?"
grep -v amdgpu.ids gpurun_out/eng2_ffn.log | tail -4
