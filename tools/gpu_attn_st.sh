# DAC halo conv: weight fragments in registers 2 / 3 / 4 steps ahead vs the LDS ring: parity tests and timing
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in default zonos_vibes_amd/var/libzonos_dacr2.so zonos_vibes_amd/var/libzonos_dacr3.so zonos_vibes_amd/var/libzonos_dacr4.so; do
  if [ $v = default ]; then unset ZMI_LIB_PATH; else export ZMI_LIB_PATH=$v; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_generate.py tests/test_dac_encode.py -k "dac or encode" >> gpurun_out/dacr_tests.log 2>&1 || exit $?
  echo "$v" >> gpurun_out/dacr.jsonl
  timeout -k 10 120 python -u tools/bench_dac.py 861 >> gpurun_out/dacr.jsonl 2>>gpurun_out/dacr.err || exit $?
  timeout -k 10 120 python -u tools/bench_dac.py 5598 >> gpurun_out/dacr.jsonl 2>>gpurun_out/dacr.err || exit $?
done
