# C3 sample under rocprofv3 for both many-row GEMM options: per-kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 1 2; do
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3prof$v -o c3 -- python3 -u tools/bench_batch.py "{\"opt_gemm_rows\": $v}" > gpurun_out/c3prof$v.log 2>&1 || exit $?
find gpurun_out/c3prof$v -name "*kernel_trace*" -delete
done
