# kernel-stats profile of the C3-shaped batch (64 slots)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3prof -o c3prof -- python tools/bench_batch.py > gpurun_out/c3prof.log 2>&1 || exit $?
find gpurun_out/c3prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/c3_kernel_stats.csv \;
rm -rf gpurun_out/c3prof
