#!/bin/bash
# One parameterised GPU-box driver (run from the repo root on the box, usually through tools/steps.sh, which
# gives every step its own time limit and stops at the first fault). Kept outputs land in gpurun_out/keep/ and are
# copied into profiles/ by hand afterwards. Subcommands:
#
#   tests [pytest args...]              GPU tests (default: the whole -m gpu suite)       -> keep/tests.log
#   bench [bench.py args...]            the headline bench                                 -> keep/bench.log
#   ab <tool.py> <tag> <arm>...         one run of `python tools/<tool.py> <arm>` per arm  -> keep/<tag>.jsonl
#                                       (an arm is the tool's argument string, shell-quoted: step_ab.py
#                                       "'[{...}, ...]'", bench_c5.py "2000 '{...}'", attn_bench.py "--rows 16 ...")
#   prof <tag> <seconds> <cmd...>       rocprofv3 --kernel-trace --stats of <cmd>          -> keep/<tag>_kernel_stats.csv
#   pmc <counter> <driver> <kernel> <bytes> <tag>
#                                       one PMC pass (tools/pmc_driver.py <driver>), summarised per launch of
#                                       <kernel> against <bytes> algorithmic bytes          -> keep/pmc_<tag>.json
#   mfma <frames> <tag>                 SQ_VALU_MFMA_BUSY_CYCLES pass over the DAC decode  -> keep/<tag>_mfma_pmc.json
#   round                               this round's profile set: bench kernel stats, fc1 FETCH, attention block
#                                       FETCH / WRITE, C5 kernel stats, DAC MFMA busy
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
K=gpurun_out/keep
mkdir -p $K
cmd="$1"
shift

prof() {  # tag seconds cmd...
  local tag=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o prof -- "$@" \
    > $K/prof_$tag.log 2>&1 || return $?
  find gpurun_out/prof_$tag -name "*kernel_stats.csv" -exec cp {} $K/${tag}_kernel_stats.csv \;
  rm -rf gpurun_out/prof_$tag
}

pmc() {  # counter driver kernel bytes tag
  timeout -s KILL 120 rocprofv3 --pmc $1 --kernel-trace --output-format csv -d gpurun_out/pmc_$5 -o pmc -- \
    python tools/pmc_driver.py $2 > $K/pmc_$5.log 2>&1 || return $?
  local f
  f=$(find gpurun_out/pmc_$5 -name "*counter_collection.csv" -print -quit)
  python tools/pmc_summary.py "$f" "$3" $4 > $K/pmc_$5.json && rm -rf gpurun_out/pmc_$5
}

mfma() {  # frames tag
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
    --output-format csv -d gpurun_out/pmc_dac -o pmc -- python tools/bench_dac.py $1 > $K/pmc_dac.log 2>&1 || return $?
  python tools/pmc_summary.py --mfma "$(find gpurun_out/pmc_dac -name "*counter_collection.csv" -print -quit)" \
    > $K/$2_mfma_pmc.json || return $?
  rm -rf gpurun_out/pmc_dac
}

case "$cmd" in
  tests)
    [ $# -eq 0 ] && set -- tests -m gpu
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "$@" \
      > $K/tests.log 2>&1
    rc=$?
    tail -3 $K/tests.log
    exit $rc
    ;;
  bench)
    timeout -k 10 600 python -u bench.py "$@" > $K/bench.log 2>&1
    rc=$?
    tail -c 600 $K/bench.log
    exit $rc
    ;;
  ab)
    tool=$1 tag=$2
    shift 2
    for arm in "$@"; do  # an arm is the tool's argument string, shell-quoted as needed
      timeout -k 10 400 bash -c "python -u tools/$tool $arm" >> $K/$tag.jsonl 2>> $K/$tag.err || exit $?
    done
    ;;
  prof) prof "$@" || exit $? ;;
  pmc) pmc "$@" || exit $? ;;
  mfma) mfma "$@" || exit $? ;;
  round)
    prof bench 500 python bench.py --no-cpu-baseline --no-hybrid --no-batch --no-c5 --no-default-cap || exit $?
    pmc FETCH_SIZE attnblk attn_block_kernel 23396352 attnblk_fetch || exit $?   # QKV + out_proj + K/V at 591
    pmc WRITE_SIZE attnblk attn_block_kernel 23396352 attnblk_write || exit $?
    pmc FETCH_SIZE fc1 "gemv_kernel<2, 4, 8, 16, 1, 3, 1>" 67158016 fc1_fetch || exit $?
    pmc FETCH_SIZE fc2 "gemv_kernel<1, 8, 16, 8, 0, 1, 1>" 33554432 fc2_fetch || exit $?
    prof c5_2000 400 python tools/bench_c5.py 2000 || exit $?
    mfma 861 dac || exit $?
    ls -la $K
    ;;
  *)
    echo "usage: tools/gpu.sh tests|bench|ab|prof|pmc|mfma|round ..." >&2
    exit 2
    ;;
esac
