#!/bin/bash
# chunked attention phase costs, back to back (timing-only builds in zonos_vibes_amd/ab/, work re-zeroed per launch)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/xcut.jsonl
for lib in default oldx cut1 cut3 cut3n cut5; do
  if [ $lib = default ]; then unset ZMI_LIB_PATH; else export ZMI_LIB_PATH=$PWD/zonos_vibes_amd/ab/lib$lib.so; fi
  for p in 1500 3200 5700; do
    timeout -k 10 120 python tools/attn_bench.py --rows 16 --pos $p --rezero >> gpurun_out/xcut.jsonl 2>> gpurun_out/xcut.err || exit 4
  done
done
