#!/bin/bash
# Round-5 A/B of the dense-pair MFMA forms (ZMI_OPT_GEMM_ROWS 3 vs 1): split-K tests, many-row GEMV timings, the
# C2 / C4 prefills, the C3 share and a C5-shaped job. Run from the repo root on the GPU box.
bash tools/steps.sh \
  "bash tools/gpu.sh tests tests/test_gpu_splitk.py" \
  "timeout -k 10 300 python tools/gemm_rows_bench.py 64,128,322 1,3 > gpurun_out/keep/grb.jsonl 2>gpurun_out/keep/grb.err" \
  "bash tools/gpu.sh ab prefill_ab.py pre_dn2 \"hybrid '[{\\\"opt:1\\\": 1}, {\\\"opt:1\\\": 3}]'\" \"transformer '[{\\\"opt:1\\\": 1}, {\\\"opt:1\\\": 3}]'\"" \
  "bash tools/gpu.sh ab bench_c3.py c3_dn2 \"'{\\\"opt:1\\\": 3}'\" \"'{\\\"opt:1\\\": 1}'\"" \
  "bash tools/gpu.sh ab bench_c5.py c5_dn \"2000 '{\\\"opt_gemm_rows\\\": 3}'\" \"2000 '{\\\"opt_gemm_rows\\\": 1}'\""
