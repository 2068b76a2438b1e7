# batched prefill (prefill_many): engine tests, C3 sample A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_generate.py tests/test_gpu_hybrid.py tests/test_gpu_c1.py tests/test_gpu_api.py > gpurun_out/pm_tests.log 2>&1 || exit $?
for o in '{"prefill_batch": false}' '{}' '{"prefill_batch": false}' '{}'; do
  timeout -k 10 300 python -u tools/bench_batch.py "$o" >> gpurun_out/pm_c3.jsonl 2>>gpurun_out/pm_c3.err || exit $?
done
