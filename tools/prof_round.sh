#!/bin/bash
# GPU-box profiling pass for this round (run from the repo root on the box):
#  1. kernel stats of the default bench (rocprofv3 --kernel-trace --stats);
#  2. HBM-traffic counter passes, one counter per pass: FETCH_SIZE on the fc1 GEMV, FETCH_SIZE and
#     WRITE_SIZE on the attention kernel (tools/pmc_driver.py);
#  3. MFMA-busy pass over the DAC decode.
# Everything kept lands in gpurun_out/keep/ (copied into profiles/ afterwards).
set -o pipefail
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
mkdir -p gpurun_out/keep
K=gpurun_out/keep
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- \
  python bench.py --no-cpu-baseline --no-hybrid --no-batch --no-c5 > $K/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $K/bench_kernel_stats.csv \;
rm -rf gpurun_out/prof
pmc() {  # counter, driver, kernel substring, algorithmic bytes, tag
  timeout -s KILL 120 rocprofv3 --pmc $1 --kernel-trace --output-format csv -d gpurun_out/pmc_$5 -o pmc -- \
    python tools/pmc_driver.py $2 > $K/pmc_$5.log 2>&1 || return $?
  f=$(find gpurun_out/pmc_$5 -name "*counter_collection.csv" -print -quit)
  python tools/pmc_summary.py "$f" "$3" $4 > $K/pmc_$5.json && rm -rf gpurun_out/pmc_$5
}
pmc FETCH_SIZE fc1 "gemv_kernel<2, 4, 8, 16, 1, 3, 1>" 67158016 fc1_fetch || exit $?
pmc FETCH_SIZE attnblk attn_block_kernel 15007744 attnblk_fetch || exit $?
pmc WRITE_SIZE attnblk attn_block_kernel 15007744 attnblk_write || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d gpurun_out/pmc_dac -o pmc -- python tools/bench_dac.py 861 > $K/pmc_dac.log 2>&1 || exit $?
python tools/pmc_summary.py --mfma "$(find gpurun_out/pmc_dac -name "*counter_collection.csv" -print -quit)" \
  > $K/dac_mfma_pmc.json || exit $?
rm -rf gpurun_out/pmc_dac
ls -la $K
