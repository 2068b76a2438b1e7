# GPU-box pass (round 3): the full -m gpu suite, sampler and long-context attention A/B, then a quick bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/step_ab.py '[{"greedy_sampler": false}, {"greedy_sampler": true}, {"greedy_sampler": false}, {"greedy_sampler": true}]' > gpurun_out/sampler_ab.jsonl 2>gpurun_out/sampler_ab.err || exit $?
for v in 1 2 1 2; do timeout -k 10 200 python -u tools/bench_c5.py 2000 $v >> gpurun_out/c5_ab.jsonl 2>>gpurun_out/c5_ab.err || exit $?; done
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
