#!/bin/bash
# C5-shaped job (8 slots, 430-frame prefix, N new frames) under rocprofv3: per-kernel time
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${1:-2000}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o c5 -- python3 -u tools/bench_c5.py $N > gpurun_out/c5prof.log 2>&1 || exit 3
find gpurun_out/c5prof -name "*kernel_trace*" -delete
