#!/bin/bash
# Diagnostic library: the fused out_proj + fc1 launch with in-kernel phase stamps (-DZMI_FFN_STAMPS)
# into zonos_vibes_amd/var/libzonos_ffnblk_stamps.so (tools/ffnblk_stamps.py reads them on the GPU).
set -e
cd "$(dirname "$0")/.."
python -m zonos_vibes_amd.build > /dev/null
mkdir -p zonos_vibes_amd/var /tmp/ffst
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc \
  -DZMI_FFN_STAMPS -c zonos_vibes_amd/csrc/zmi_ffnblk.hip -o /tmp/ffst/zmi_ffnblk.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls zonos_vibes_amd/build/*.o | grep -v zmi_ffnblk) \
  /tmp/ffst/zmi_ffnblk.o -o zonos_vibes_amd/var/libzonos_ffnblk_stamps.so
