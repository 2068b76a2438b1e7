#!/bin/bash
# Diagnostic library: the GEMV kernels with in-kernel phase stamps (-DZMI_GEMV_STAMPS) into
# zonos_vibes_amd/var/libzonos_gemv_stamps.so (tools/gemv_stamps.py, tools/hybrid_stamps.py read them on the GPU;
# the hybrid's mamba block stamps its step role too).
set -e
cd "$(dirname "$0")/.."
python -m zonos_vibes_amd.build > /dev/null
mkdir -p zonos_vibes_amd/var /tmp/gst
objs=""
STAMPED="zmi_gemv zmi_gemv_e0 zmi_gemv_e1 zmi_gemv_e2 zmi_gemv_e3 zmi_gemv_e4 zmi_gemv_e5 zmi_mambablk"
for f in $STAMPED; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc \
    -DZMI_GEMV_STAMPS -c zonos_vibes_amd/csrc/$f.hip -o /tmp/gst/$f.o &
  objs="$objs /tmp/gst/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls zonos_vibes_amd/build/*.o | grep -v -e zmi_gemv -e zmi_mambablk) $objs \
  -o zonos_vibes_amd/var/libzonos_gemv_stamps.so
