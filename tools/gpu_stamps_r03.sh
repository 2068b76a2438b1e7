set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-hybrid --no-batch --no-c5 > gpurun_out/r03h_bench_quick.log 2>&1 || exit $?
for p in 300 591 900; do
ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_ffnblk_stamps.so timeout -k 10 120 python -u tools/ffnblk_stamps.py --pos $p >> gpurun_out/r03h_ffn_stamps.jsonl 2>gpurun_out/r03h_ffn_stamps.err || exit $?
ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_attnblk_stamps.so timeout -k 10 120 python -u tools/attnblk_stamps.py --pos $p >> gpurun_out/r03h_attn_stamps.jsonl 2>gpurun_out/r03h_attn_stamps.err || exit $?
done
