#!/bin/bash
# Build libzonos_hip variants that differ only in the attention chunk size (ZMI_ATTN_NWC waves of
# 32 keys per workgroup) into zonos_vibes_amd/var/ (tools/attn_variants.sh times them on the GPU).
set -e
cd "$(dirname "$0")/.."
python -m zonos_vibes_amd.build > /dev/null
mkdir -p zonos_vibes_amd/var
if [ "$1" = "--stamps" ]; then
  shift
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc \
    -DZMI_ATTN_STAMPS ${1:+-DZMI_ATTN_NWC=$1} -c zonos_vibes_amd/csrc/zmi_attn.hip -o /tmp/attn_st.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls zonos_vibes_amd/build/*.o | grep -v '/zmi_attn.o$') \
    /tmp/attn_st.o -o zonos_vibes_amd/var/libzonos_attn_stamps.so
  exit 0
fi
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc \
    -DZMI_ATTN_NWC=$n -c zonos_vibes_amd/csrc/zmi_attn.hip -o /tmp/attn$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls zonos_vibes_amd/build/*.o | grep -v '/zmi_attn.o$') \
    /tmp/attn$n.o -o zonos_vibes_amd/var/libzonos_nwc$n.so
done
