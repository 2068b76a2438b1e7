set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attnffn.py > gpurun_out/af_test.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/step_ab.py '[{"attn_ffn": false}, {"attn_ffn": true, "opt_af_depth": 3}, {"attn_ffn": true, "opt_af_depth": 0}, {"attn_ffn": true, "opt_af_depth": 3, "opt_af_delay": 1}, {"attn_ffn": true, "opt_af_depth": 3, "opt_af_delay": 2}, {"attn_ffn": true, "opt_af_depth": 3, "opt_af_delay": 4}, {"attn_ffn": true, "opt_af_depth": 6, "opt_af_delay": 2}, {"attn_ffn": false}]' > gpurun_out/af_ab.jsonl 2>gpurun_out/af_ab.err || exit $?
for d in 0 2; do
ZMI_AF_DELAY=$d ZMI_LIB_PATH=zonos_vibes_amd/var/libzonos_attnffn_stamps.so timeout -k 10 120 python -u tools/attnffn_stamps.py --pos 591 >> gpurun_out/af_stamps.jsonl 2>gpurun_out/af_stamps.err || exit $?
done
