# C3 sample A/B: out_proj split-K upper row bound (64 vs none)
set -o pipefail
cd $GRAFT_REPO_ROOT
for o in '{"splitk_o_max_rows": 64}' '{"splitk_o_max_rows": 100000}' '{"splitk_o_max_rows": 64}' '{"splitk_o_max_rows": 100000}'; do
  timeout -k 10 300 python -u tools/bench_batch.py "$o" >> gpurun_out/skmax_c3.jsonl 2>>gpurun_out/skmax_c3.err || exit $?
done
