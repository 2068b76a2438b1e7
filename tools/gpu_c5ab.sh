# C5-shaped A/B at 4 and 8 rows: fused QKV + attention forms vs separate launches
set -o pipefail
cd $GRAFT_REPO_ROOT
for sl in 2 4; do
for o in '{}' '{"attn_block_rows": 2}' '{"attn_forms": ["split"]}' '{"attn_block_rows": 4}' '{}' '{"attn_block_rows": 2}' '{"attn_forms": ["split"]}' '{"attn_block_rows": 4}'; do
  timeout -k 10 200 python -u tools/bench_c5.py 1000 "$o" $sl >> gpurun_out/abr2_c5.jsonl 2>>gpurun_out/abr2_c5.err || exit $?
done
done
