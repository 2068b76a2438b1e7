#!/bin/bash
# Diagnostic library: the fused QKV + attention launch with in-kernel phase stamps for both roles
# (-DZMI_ATTN_STAMPS -DZMI_GEMV_STAMPS) into zonos_vibes_amd/var/libzonos_attnblk_stamps${TAG}.so
# (tools/attnblk_stamps.py reads them on the GPU). Extra defines (e.g. -DZMI_LN_STAMP=1: the projection role's
# slot 7 after the LayerNorm's first pass) go in $EXTRA, the library name suffix in $TAG.
set -e
cd "$(dirname "$0")/.."
python -m zonos_vibes_amd.build > /dev/null
mkdir -p zonos_vibes_amd/var /tmp/abst
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc \
  -DZMI_ATTN_STAMPS -DZMI_GEMV_STAMPS $EXTRA -c zonos_vibes_amd/csrc/zmi_attnblk.hip -o /tmp/abst/zmi_attnblk${TAG}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls zonos_vibes_amd/build/*.o | grep -v zmi_attnblk) \
  /tmp/abst/zmi_attnblk${TAG}.o -o zonos_vibes_amd/var/libzonos_attnblk_stamps${TAG}.so
