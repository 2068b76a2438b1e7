#!/bin/bash
# the wide chunk-split form: one workgroup per CU (default) against co-resident workgroups (libcoloc.so)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/s24b.jsonl
for lib in default coloc default coloc; do
  if [ $lib = default ]; then unset ZMI_LIB_PATH; else export ZMI_LIB_PATH=$PWD/zonos_vibes_amd/ab/lib$lib.so; fi
  timeout -k 10 200 python -u tools/bench_long.py "{\"ab_tag\": \"$lib\"}" >> gpurun_out/s24b.jsonl 2>> gpurun_out/s24b.err || exit 4
done
