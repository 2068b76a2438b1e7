# GPU-box pass (round 3): the default bench (all widened lines), then the profiling pass (tools/prof_round.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
bash tools/prof_round.sh || exit $?
