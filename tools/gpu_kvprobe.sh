#!/bin/bash
# K / V read probe (tools/kv_probe.py), 16 rows: K only, V^T only, V^T linear, both
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/kvprobe3.jsonl
for p in 1500 3200 5700; do
  timeout -k 10 240 python tools/kv_probe.py --rows 16 --pos $p --modes 3,4,6,7 --occ 3,6,8 >> gpurun_out/kvprobe3.jsonl 2>> gpurun_out/kvprobe.err || exit 4
done
