#!/bin/bash
# two-launch attention: load order x merge width builds (zonos_vibes_amd/ab/), 16 rows
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/two_ab.jsonl
for lib in default m4; do
  if [ $lib = default ]; then unset ZMI_LIB_PATH; else export ZMI_LIB_PATH=$PWD/zonos_vibes_amd/ab/lib$lib.so; fi
  for p in 1500 3200; do
    timeout -k 10 120 python tools/attn_bench.py --rows 16 --pos $p --variant 2 >> gpurun_out/two_ab.jsonl 2>> gpurun_out/two_ab.err || exit 4
  done
done
