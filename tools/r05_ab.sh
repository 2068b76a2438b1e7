#!/bin/bash
# Round-5 GPU-box A/B runs, one subcommand each (run from the repo root on the box; outputs in gpurun_out/keep/,
# copied into profiles/r05_* by hand):
#   dense     ZMI_OPT_GEMM_ROWS 3 vs 1 (dense-pair MFMAs): split-K tests, many-row GEMM timings, C2 / C4 prefills,
#             the C3 share, a C5-shaped job
#   stage     ZMI_OPT_SPLITK_STAGE 1 vs 0 (row tiles per LDS stage): the same set with the split-K timings
#   ssd       ZMI_OPT_SCAN_PQ 0 vs 4 (the SSD prefill scan): scan oracle tests, C4 prefill A/B (times only: the forms
#             differ in fp32 rounding), its kernel stats
#   oproj24   the fused out_proj role in the 24-chunk form (engine attn_oproj_wide): tests, the 30 s batch-1 line
#   pmc_ssd   one PMC pass (LDS / wait counters) over the C4 prefill
#   pf        the separate attention launch's prefetch workgroups (engine attn_prefetch_blocks 128 / 256 / 384): the
#             C3 share and a C5-shaped job, arms alternating
case "$1" in
  dense)
    bash tools/steps.sh \
      "bash tools/gpu.sh tests tests/test_gpu_splitk.py" \
      "timeout -k 10 300 python tools/gemm_rows_bench.py 64,128,322 1,3 > gpurun_out/keep/grb.jsonl 2>gpurun_out/keep/grb.err" \
      "bash tools/gpu.sh ab prefill_ab.py pre_dn2 \"hybrid '[{\\\"opt:1\\\": 1}, {\\\"opt:1\\\": 3}]'\" \"transformer '[{\\\"opt:1\\\": 1}, {\\\"opt:1\\\": 3}]'\"" \
      "bash tools/gpu.sh ab bench_c3.py c3_dn2 \"'{\\\"opt:1\\\": 3}'\" \"'{\\\"opt:1\\\": 1}'\"" \
      "bash tools/gpu.sh ab bench_c5.py c5_dn \"2000 '{\\\"opt_gemm_rows\\\": 3}'\" \"2000 '{\\\"opt_gemm_rows\\\": 1}'\"" ;;
  stage)
    bash tools/steps.sh \
      "bash tools/gpu.sh tests tests/test_gpu_splitk.py" \
      "timeout -k 10 300 python tools/splitk_bench.py 16,128,322 '[{\"17\": 1}, {\"17\": 0}]' > gpurun_out/keep/skb.jsonl 2>gpurun_out/keep/skb.err" \
      "bash tools/gpu.sh ab prefill_ab.py pre_st \"hybrid '[{\\\"opt:17\\\": 1}, {\\\"opt:17\\\": 0}]'\" \"transformer '[{\\\"opt:17\\\": 1}, {\\\"opt:17\\\": 0}]'\"" \
      "bash tools/gpu.sh ab bench_c3.py c3_st \"'{\\\"opt:17\\\": 1}'\" \"'{\\\"opt:17\\\": 0}'\"" \
      "bash tools/gpu.sh ab bench_c5.py c5_st \"2000 '{\\\"opt_splitk_stage\\\": 1}'\" \"2000 '{\\\"opt_splitk_stage\\\": 0}'\"" ;;
  ssd)
    bash tools/steps.sh \
      "bash tools/gpu.sh tests tests/test_gpu_hybrid.py -k scan" \
      "bash tools/gpu.sh ab prefill_ab.py pre_ssd \"hybrid '[{\\\"opt:15\\\": 4}, {\\\"opt:15\\\": 0}]' 7 nocheck\"" \
      "bash tools/gpu.sh prof hybpre_ssd 200 python tools/prefill_ab.py hybrid '[{\"opt:15\": 0}]' 5" ;;
  oproj24)
    bash tools/steps.sh \
      "bash tools/gpu.sh tests tests/test_gpu_attnblk.py tests/test_gpu_kernels.py tests/test_gpu_splitk.py -k \"attn_block or production_shapes or splitk\"" \
      "bash tools/gpu.sh ab bench_long.py long_oproj \"'{\\\"attn_oproj_wide\\\": true}'\" \"'{\\\"attn_oproj_wide\\\": false}'\" \"'{\\\"attn_oproj_wide\\\": true}'\"" ;;
  pf)
    k=gpurun_out/keep
    for arm in 256 128 384 256 128 384; do
      timeout -k 10 300 python -u tools/bench_c3.py "{\"attn_prefetch_blocks\": $arm}" >> $k/c3_pf.jsonl 2>> $k/c3_pf.err || exit $?
    done
    for arm in 128 256 128 256; do
      timeout -k 10 300 python -u tools/bench_c5.py 2000 "{\"attn_prefetch_blocks\": $arm}" >> $k/c5_pf.jsonl 2>> $k/c5_pf.err || exit $?
    done ;;
  pmc_ssd)
    cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}" || exit 1
    mkdir -p gpurun_out/keep
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES \
      --kernel-trace --output-format csv -d gpurun_out/pmc_ssd -o pmc -- python tools/prefill_ab.py hybrid '[{"opt:15": 0}]' 1 \
      > gpurun_out/keep/pmc_ssd.log 2>&1 || exit $?
    python tools/pmc_summary.py --per-kernel "$(find gpurun_out/pmc_ssd -name '*counter_collection.csv' -print -quit)" \
      > gpurun_out/keep/pmc_ssd.json && rm -rf gpurun_out/pmc_ssd ;;
  *)
    echo "usage: tools/r05_ab.sh dense|stage|ssd|oproj24|pmc_ssd" >&2
    exit 2 ;;
esac
