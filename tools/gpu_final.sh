# round-3 final GPU pass: smoke(), the whole -m gpu suite, then the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
