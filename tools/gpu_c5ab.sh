# C2 step A/B: prefetch role sizes with the separate out_proj / fc1 launches
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/step_ab.py '[{"prefetch_blocks": 256, "prefetch_fc1_mb": 8}, {"prefetch_blocks": 256, "prefetch_fc1_mb": 4}, {"prefetch_blocks": 256, "prefetch_fc1_mb": 16}, {"prefetch_blocks": 384, "prefetch_fc1_mb": 8}, {"prefetch_blocks": 512, "prefetch_fc1_mb": 8}, {"prefetch_blocks": 512, "prefetch_fc1_mb": 16}, {"prefetch_blocks": 128, "prefetch_fc1_mb": 4}, {"prefetch_blocks": 256, "prefetch_fc1_mb": 8}]' > gpurun_out/pf_ab3.jsonl 2>gpurun_out/pf_ab3.err || exit $?
