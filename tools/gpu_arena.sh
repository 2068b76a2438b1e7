#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/arena_ab.jsonl
for p in 1 2; do
  timeout -k 10 300 python -u tools/arena_ab.py | sed "s/^{/{\"proc\": $p, /" >> gpurun_out/arena_ab.jsonl 2>> gpurun_out/arena_ab.err || exit 5
done
cat gpurun_out/arena_ab.jsonl
