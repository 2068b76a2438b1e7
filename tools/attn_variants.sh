set -o pipefail
mkdir -p gpurun_out
for n in ${NWCS:-4 8 16}; do
  export ZMI_LIB_PATH=$PWD/zonos_vibes_amd/var/libzonos_nwc$n.so
  echo "== nwc $n" >> gpurun_out/av.log
  timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k attention --timeout 120 --timeout-method thread >> gpurun_out/av.log 2>&1 || exit 3
  for s in 1 64; do for p in 300 591; do
    timeout -k 10 120 python tools/kernel_bench.py --slots $s --pos $p --reps 3 2>/dev/null | grep attention >> gpurun_out/av.log || exit 4
  done; done
done
