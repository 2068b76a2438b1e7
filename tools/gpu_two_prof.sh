#!/bin/bash
# per-launch durations (rocprofv3 kernel trace) of the two-launch attention: full and cut after M_j + V^T
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/twoprof2 -o run -- python3 tools/attn_bench.py --rows 16 --pos 3200 --variant 2 > gpurun_out/twoprof2.log 2>&1 || exit 3
ZMI_LIB_PATH=$PWD/zonos_vibes_amd/ab/libbcut.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/twoprofc -o run -- python3 tools/attn_bench.py --rows 16 --pos 3200 --variant 2 --rezero > gpurun_out/twoprofc.log 2>&1 || exit 4
