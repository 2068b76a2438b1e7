#!/bin/bash
# Diagnostic library: the fused attention + out_proj + fc1 launch with in-kernel phase stamps
# (-DZMI_ATTNFFN_STAMPS) into zonos_vibes_amd/var/libzonos_attnffn_stamps.so (tools/attnffn_stamps.py).
set -e
cd "$(dirname "$0")/.."
python -m zonos_vibes_amd.build > /dev/null
mkdir -p zonos_vibes_amd/var /tmp/afst
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc \
  -DZMI_ATTNFFN_STAMPS -c zonos_vibes_amd/csrc/zmi_attnffn.hip -o /tmp/afst/zmi_attnffn.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls zonos_vibes_amd/build/*.o | grep -v zmi_attnffn) \
  /tmp/afst/zmi_attnffn.o -o zonos_vibes_amd/var/libzonos_attnffn_stamps.so
