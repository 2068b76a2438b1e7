#!/bin/bash
# One PMC pass over the C4 prefill with the quadratic (SSD) scan: LDS instructions / bank conflicts / waits and
# wave cycles per kernel (tools/pmc_summary.py --per-kernel).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}" || exit 1
mkdir -p gpurun_out/keep
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_ssd -o pmc -- python tools/prefill_ab.py hybrid '[{"opt:15": 0}]' 1 \
  > gpurun_out/keep/pmc_ssd.log 2>&1 || exit $?
python tools/pmc_summary.py --per-kernel "$(find gpurun_out/pmc_ssd -name '*counter_collection.csv' -print -quit)" \
  > gpurun_out/keep/pmc_ssd.json && rm -rf gpurun_out/pmc_ssd
