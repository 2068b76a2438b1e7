#!/bin/bash
# attention phase stamps, 16 rows, back to back (last of 6 launches over rotating caches), one launch vs pair
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/xst.jsonl
for v in 1 2; do
  echo "{\"variant\": $v}" >> gpurun_out/xst.jsonl
  ZMI_LIB_PATH=$PWD/zonos_vibes_amd/ab/libst.so ATTN_VARIANT=$v ATTN_SLOTS=8 ATTN_ROTATE=6 timeout -k 10 200 \
    python tools/attn_stamps.py 1500 3200 >> gpurun_out/xst.jsonl 2>> gpurun_out/xst.err || exit 3
done
