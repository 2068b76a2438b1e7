#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layer_engine.py > gpurun_out/eng5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/eng5_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/eng5_tests.log | head; exit $rc; fi
timeout -k 10 400 python -u tools/step_ab.py '[{"layer_engine": false}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 8, "opt_eng_hold": 1}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 2, "opt_eng_hold": 1}, {"layer_engine": true, "opt_eng_fly": 8, "opt_eng_thin": 8, "opt_eng_hold": 0}, {"layer_engine": true, "opt_eng_fly": 4, "opt_eng_thin": 4, "opt_eng_hold": 1}, {"layer_engine": true, "opt_eng_fly": 6, "opt_eng_thin": 6, "opt_eng_hold": 1}]' > gpurun_out/eng5_ab.log 2>&1; echo "ab rc=$?"
grep -v amdgpu.ids gpurun_out/eng5_ab.log | tail -6
timeout -k 10 200 python -u tools/layer_engine_stamps.py 13 8 8 > gpurun_out/eng5_stamps.log 2>&1; echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/eng5_stamps.log | tail -1
