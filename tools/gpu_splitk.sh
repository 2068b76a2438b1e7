# split-K fc2 / out_proj + fused LayerNorm: bit-identity, batch invariance through the engine, C3 / C5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_splitk.py tests/test_gpu_scale.py tests/test_gpu_generate.py > gpurun_out/splitk_tests.log 2>&1 || exit $?
for o in '{"splitk_o_rows": 0}' '{"splitk_o_rows": 16}' '{"splitk_o_rows": 0}' '{"splitk_o_rows": 16}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 1000 "$o" >> gpurun_out/splitko_c5.jsonl 2>>gpurun_out/splitko_c5.err || exit $?
done
for o in '{"splitk_o_rows": 0}' '{"splitk_o_rows": 16}'; do
  timeout -k 10 300 python -u tools/bench_batch.py "$o" >> gpurun_out/splitko_c3.jsonl 2>>gpurun_out/splitko_c3.err || exit $?
done
