#!/bin/bash
# DAC profiling pass (run from the repo root on the GPU box): kernel stats of tools/bench_dac.py, then one
# MFMA-busy counter pass. Outputs land in gpurun_out/dac/ (copied into profiles/ afterwards).
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
K=gpurun_out/dac
mkdir -p $K
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dprof -o prof -- \
  python tools/bench_dac.py 861 > $K/bench_dac.log 2>&1 || exit $?
find gpurun_out/dprof -name "*kernel_stats.csv" -exec cp {} $K/dac_kernel_stats.csv \;
rm -rf gpurun_out/dprof
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d gpurun_out/pmc_dac -o pmc -- python tools/bench_dac.py 861 > $K/pmc_dac.log 2>&1 || exit $?
python tools/pmc_summary.py --mfma "$(find gpurun_out/pmc_dac -name "*counter_collection.csv" -print -quit)" \
  > $K/dac_mfma_pmc.json || exit $?
rm -rf gpurun_out/pmc_dac
