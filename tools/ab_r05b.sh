#!/bin/bash
# Round-5 second batch: the fused out_proj role in the 24-chunk split form (tests + the 30 s batch-1 line on / off)
# and the rotated row-tile order of the many-row / split-K GEMMs (ZMI_OPT_GEMM_ROWS 7 vs 3).
bash tools/steps.sh \
  "bash tools/gpu.sh tests tests/test_gpu_attnblk.py tests/test_gpu_kernels.py tests/test_gpu_splitk.py -k \"attn_block or production_shapes or splitk\"" \
  "bash tools/gpu.sh ab bench_long.py long_oproj \"'{\\\"attn_oproj_wide\\\": true}'\" \"'{\\\"attn_oproj_wide\\\": false}'\" \"'{\\\"attn_oproj_wide\\\": true}'\"" \
  "timeout -k 10 300 python tools/gemm_rows_bench.py 64,128,322 3,7 > gpurun_out/keep/grb_rot.jsonl 2>gpurun_out/keep/grb_rot.err" \
  "bash tools/gpu.sh ab prefill_ab.py pre_rot \"hybrid '[{\\\"opt:1\\\": 3}, {\\\"opt:1\\\": 7}]'\" \"transformer '[{\\\"opt:1\\\": 3}, {\\\"opt:1\\\": 7}]'\"" \
  "bash tools/gpu.sh ab bench_c3.py c3_rot \"'{\\\"opt:1\\\": 7}'\" \"'{\\\"opt:1\\\": 3}'\" \"'{\\\"opt:1\\\": 7}'\""
