# C5 share under rocprofv3: per-kernel time at 16 rows (8 slots); $1 = engine options JSON
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o c5 -- python3 -u tools/bench_c5.py 1000 "$1" > gpurun_out/c5prof.log 2>&1 || exit $?
find gpurun_out/c5prof -name "*kernel_trace*" -delete
