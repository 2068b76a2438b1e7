#!/bin/bash
# K / V read probe against the attention kernel (tools/kv_probe.py, tools/attn_bench.py), 16 rows.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/kvprobe.jsonl
for p in 1500 3200; do
  timeout -k 10 180 python tools/attn_bench.py --rows 16 --pos $p >> gpurun_out/kvprobe.jsonl 2>> gpurun_out/kvprobe.err || exit 3
  timeout -k 10 240 python tools/kv_probe.py --rows 16 --pos $p >> gpurun_out/kvprobe.jsonl 2>> gpurun_out/kvprobe.err || exit 4
done
