#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layer_engine.py > gpurun_out/eng6_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/eng6_tests.log; if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/eng6_tests.log | head; exit $rc; fi
timeout -k 10 400 python -u tools/step_ab.py '[{"layer_engine": false}, {"layer_engine": true, "opt_eng_pf": 0}, {"layer_engine": true, "opt_eng_pf": 1}, {"layer_engine": true, "opt_eng_pf": 1, "opt_eng_delay": 1000}, {"layer_engine": true, "opt_eng_pf": 1, "opt_eng_delay": 2000}, {"layer_engine": true, "opt_eng_pf": 1, "opt_eng_thin": 8}, {"layer_engine": true, "opt_eng_pf": 0, "opt_eng_delay": 1500}]' > gpurun_out/eng6_ab.log 2>&1; echo "ab rc=$?"
grep -v amdgpu.ids gpurun_out/eng6_ab.log | tail -7
timeout -k 10 200 python -u tools/layer_engine_stamps.py 13 8 2 > gpurun_out/eng6_stamps.log 2>&1; echo "stamps rc=$?"
grep -v amdgpu.ids gpurun_out/eng6_stamps.log | tail -1
