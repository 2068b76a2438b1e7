#!/bin/bash
# prefetch roles of the decode GEMVs (fc1 -> fc2 head, fc2 -> next QKV): GEMV parity, then the C2 step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k gemv > gpurun_out/gpf_tests.log 2>&1 || exit 3
timeout -k 10 600 python -u tools/step_ab.py '[{}, {"fc2_prefetch_mb": 12}, {"fc1_prefetch_mb": 8}, {"fc1_prefetch_mb": 16}, {"fc1_prefetch_mb": 8, "fc2_prefetch_mb": 12}, {"fc2_prefetch_mb": 12, "gemv_prefetch_blocks": 256}, {}, {"fc2_prefetch_mb": 12}]' > gpurun_out/gpf.jsonl 2> gpurun_out/gpf.err || exit 4
