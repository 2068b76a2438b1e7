#!/bin/bash
# Diagnostic library: the fused QKV + attention launch with in-kernel phase stamps for both roles
# (-DZMI_ATTN_STAMPS -DZMI_GEMV_STAMPS) into zonos_vibes_amd/var/libzonos_attnblk_stamps.so
# (tools/attnblk_stamps.py reads them on the GPU).
set -e
cd "$(dirname "$0")/.."
python -m zonos_vibes_amd.build > /dev/null
mkdir -p zonos_vibes_amd/var /tmp/abst
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc \
  -DZMI_ATTN_STAMPS -DZMI_GEMV_STAMPS -c zonos_vibes_amd/csrc/zmi_attnblk.hip -o /tmp/abst/zmi_attnblk.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls zonos_vibes_amd/build/*.o | grep -v zmi_attnblk) \
  /tmp/abst/zmi_attnblk.o -o zonos_vibes_amd/var/libzonos_attnblk_stamps.so
