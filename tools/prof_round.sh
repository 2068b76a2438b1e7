#!/bin/bash
# GPU-box profiling pass: kernel stats of the default bench + an MFMA counter pass over the DAC paths.
# Big per-dispatch trace CSVs are deleted on the box (gpurun copies back at most 64 MiB); the stats
# and the counter rows are kept under gpurun_out/keep/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/keep
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python bench.py --no-cpu-baseline > gpurun_out/keep/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/keep/bench_kernel_stats.csv \;
rm -rf gpurun_out/prof
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d gpurun_out/pmc_dac -o pmc -- python tools/bench_dac.py 861 > gpurun_out/keep/pmc_dac.log 2>&1 || exit $?
find gpurun_out/pmc_dac -name "*counter_collection.csv" -exec cp {} gpurun_out/keep/dac_counters.csv \;
rm -rf gpurun_out/pmc_dac
ls -la gpurun_out/keep
