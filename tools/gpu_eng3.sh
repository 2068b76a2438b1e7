#!/bin/bash
# layer engine with a loader wave: tests, then fly/thin sweep (C2 step), stamps
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_layer_engine.py > gpurun_out/eng3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL" gpurun_out/eng3_tests.log | head -10
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/eng3_tests.log | head -20; tail -5 gpurun_out/eng3_tests.log; exit $rc; fi
timeout -k 10 400 python -u tools/step_ab.py '[{"layer_engine": false}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 1}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 2}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 4}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 8}, {"layer_engine": true, "opt_eng_fly": 4, "opt_eng_thin": 1}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 1}]' > gpurun_out/eng3_ab.log 2>&1; echo "ab rc=$?"
grep -v amdgpu.ids gpurun_out/eng3_ab.log | tail -8
timeout -k 10 300 python -u tools/layer_engine_stamps.py 13 > gpurun_out/eng3_stamps.log 2>&1; echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/eng3_stamps.log | tail -2
