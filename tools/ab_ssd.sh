#!/bin/bash
# Round-5 check of the quadratic (SSD) Mamba2 prefill form (ZMI_OPT_SCAN_PQ 0) against the 4-workgroup scan: the
# scan oracle tests, then the C4 prefill A/B (prefill logits must match within the arms' own tolerance: the forms
# differ in fp32 rounding, so the A/B compares times only).
bash tools/steps.sh \
  "bash tools/gpu.sh tests tests/test_gpu_hybrid.py -k scan" \
  "bash tools/gpu.sh ab prefill_ab.py pre_ssd \"hybrid '[{\\\"opt:15\\\": 4}, {\\\"opt:15\\\": 0}]' 7 nocheck\"" \
  "bash tools/gpu.sh prof hybpre_ssd 200 python tools/prefill_ab.py hybrid '[{\"opt:15\": 0}]' 5"
