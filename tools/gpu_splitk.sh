# split-K fc2 + fused LayerNorm: bit-identity, batch invariance through the engine, C3 / C5 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_splitk.py tests/test_gpu_scale.py tests/test_gpu_generate.py > gpurun_out/splitk_tests.log 2>&1 || exit $?
for o in '{"splitk_rows": 0}' '{"splitk_rows": 16}' '{"splitk_rows": 0}' '{"splitk_rows": 16}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 1000 "$o" >> gpurun_out/splitk_c5b.jsonl 2>>gpurun_out/splitk_c5b.err || exit $?
done
timeout -k 10 300 python -u tools/bench_batch.py > gpurun_out/splitk_c3b.jsonl 2>gpurun_out/splitk_c3b.err || exit $?
