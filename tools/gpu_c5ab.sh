# C5 / C3 A/B: out_proj split-K (+ fused ln2) with the 16-row steps on separate QKV + attention launches
set -o pipefail
cd $GRAFT_REPO_ROOT
for o in '{"splitk_o_rows": 0}' '{"splitk_o_rows": 16}' '{"splitk_o_rows": 0}' '{"splitk_o_rows": 16}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 1000 "$o" >> gpurun_out/sko2_c5.jsonl 2>>gpurun_out/sko2_c5.err || exit $?
done
for o in '{"splitk_o_rows": 0}' '{"splitk_o_rows": 16}' '{"splitk_o_rows": 0}' '{"splitk_o_rows": 16}'; do
  timeout -k 10 300 python -u tools/bench_batch.py "$o" >> gpurun_out/sko2_c3.jsonl 2>>gpurun_out/sko2_c3.err || exit $?
done
