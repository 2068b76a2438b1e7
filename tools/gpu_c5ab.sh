# C2 step A/B (ffn_block at 2 rows), then the C5 share at full length with the default plan
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/step_ab.py '[{"ffn_block": false}, {"ffn_block": true}, {"ffn_block": false}, {"ffn_block": true}]' > gpurun_out/ffn2_ab.jsonl 2>gpurun_out/ffn2_ab.err || exit $?
timeout -k 10 200 python -u tools/bench_c5.py > gpurun_out/c5_full.jsonl 2>gpurun_out/c5_full.err || exit $?
