# many-row GEMM phase stamps at 128 rows (64 slots)
set -o pipefail
cd $GRAFT_REPO_ROOT
ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_gemv_stamps.so timeout -k 10 200 python -u tools/gemm_rows_stamps.py --slots 64 --layers 1 > gpurun_out/grst2.jsonl 2>gpurun_out/grst2.err || exit $?
