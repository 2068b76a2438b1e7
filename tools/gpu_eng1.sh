#!/bin/bash
# engine round-4 pass 1: engine timing variants, C2 step A/B, engine tests
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ffn_engine_bench.py 20 0,1,2,1 > gpurun_out/eng_bench2.log 2>&1; echo "bench rc=$?"
cat gpurun_out/eng_bench2.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/step_ab.py '[{"ffn_engine": false}, {"ffn_engine": true}, {"ffn_engine": true, "opt_eng_start": 0}, {"ffn_engine": false}, {"ffn_engine": true}]' > gpurun_out/eng_step_ab.log 2>&1; echo "step_ab rc=$?"
grep -v amdgpu.ids gpurun_out/eng_step_ab.log | tail -8
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_kernels.py -k "engine or v1025 or sampler" > gpurun_out/eng_tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/eng_tests.log
