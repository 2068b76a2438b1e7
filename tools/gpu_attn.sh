# long-context attention vs the KV capacity (V^T row stride): same positions, tight and loose smax
set -o pipefail
cd $GRAFT_REPO_ROOT
for rp in "16 1500 1576" "16 1500 6000" "16 1500 12000" "16 3200 3280" "16 3200 12000" "2 1500 1576" "2 1500 12000"; do
  set -- $rp
  timeout -k 10 120 python -u tools/attn_bench.py --rows $1 --pos $2 --smax $3 --layers 8 >> gpurun_out/attn_bench3.jsonl 2>>gpurun_out/attn_bench3.err || exit $?
done
