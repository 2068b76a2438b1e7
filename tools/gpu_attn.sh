# long-context chunked attention: parity tests, microbench at 16 rows, C5 share
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_attnblk.py tests/test_gpu_attnffn.py -k "attn or attention" > gpurun_out/attnq_tests.log 2>&1 || exit $?
for rp in "16 1500" "16 3200" "16 5000" "2 1500" "128 1000"; do
  set -- $rp
  timeout -k 10 120 python -u tools/attn_bench.py --rows $1 --pos $2 --layers 8 >> gpurun_out/attnq_bench.jsonl 2>>gpurun_out/attnq_bench.err || exit $?
done
timeout -k 10 200 python -u tools/bench_c5.py 1000 '{}' >> gpurun_out/attnq_c5.jsonl 2>>gpurun_out/attnq_c5.err || exit $?
timeout -k 10 300 python -u tools/bench_c5.py 5168 '{}' >> gpurun_out/attnq_c5.jsonl 2>>gpurun_out/attnq_c5.err || exit $?
