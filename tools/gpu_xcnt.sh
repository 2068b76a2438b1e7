#!/bin/bash
# counted block-maxima exchange (default) against the granule exchange (zonos_vibes_amd/ab/liboldx.so): attention
# parity tests, then the long-context attention timing at both.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_attnblk.py > gpurun_out/xcnt_tests.log 2>&1 || exit 3
: > gpurun_out/xcnt.jsonl
for lib in default ab/liboldx.so; do
  if [ $lib = default ]; then unset ZMI_LIB_PATH; else export ZMI_LIB_PATH=$PWD/zonos_vibes_amd/$lib; fi
  for rp in "16 1500" "16 3200" "16 5700" "2 3200" "128 1000" "8 3200"; do
    set -- $rp
    timeout -k 10 120 python tools/attn_bench.py --rows $1 --pos $2 >> gpurun_out/xcnt.jsonl 2>> gpurun_out/xcnt.err || exit 4
  done
done
