# DAC halo conv A-ring depth 2 / 3 / 4: parity tests and decode timing
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in default zonos_vibes_amd/var/libzonos_dacns3.so zonos_vibes_amd/var/libzonos_dacns4.so; do
  if [ $v = default ]; then unset ZMI_LIB_PATH; else export ZMI_LIB_PATH=$v; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generate.py tests/test_dac_encode.py -k "dac or encode" >> gpurun_out/dacns_tests.log 2>&1 || exit $?
  echo "$v" >> gpurun_out/dacns.jsonl
  timeout -k 10 120 python -u tools/bench_dac.py 861 >> gpurun_out/dacns.jsonl 2>>gpurun_out/dacns.err || exit $?
  timeout -k 10 120 python -u tools/bench_dac.py 5598 >> gpurun_out/dacns.jsonl 2>>gpurun_out/dacns.err || exit $?
done
