#!/bin/bash
# Round-5 A/B of zmi_gemv_splitk's multi-tile stages (ZMI_OPT_SPLITK_STAGE 1 vs 0): tests, GEMM timings, prefills,
# the C3 share and a C5-shaped job.
bash tools/steps.sh \
  "bash tools/gpu.sh tests tests/test_gpu_splitk.py" \
  "timeout -k 10 300 python tools/splitk_bench.py 16,128,322 '[{\"17\": 1}, {\"17\": 0}]' > gpurun_out/keep/skb.jsonl 2>gpurun_out/keep/skb.err" \
  "bash tools/gpu.sh ab prefill_ab.py pre_st \"hybrid '[{\\\"opt:17\\\": 1}, {\\\"opt:17\\\": 0}]'\" \"transformer '[{\\\"opt:17\\\": 1}, {\\\"opt:17\\\": 0}]'\"" \
  "bash tools/gpu.sh ab bench_c3.py c3_st \"'{\\\"opt:17\\\": 1}'\" \"'{\\\"opt:17\\\": 0}'\"" \
  "bash tools/gpu.sh ab bench_c5.py c5_st \"2000 '{\\\"opt_splitk_stage\\\": 1}'\" \"2000 '{\\\"opt_splitk_stage\\\": 0}'\""
