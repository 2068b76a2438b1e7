#!/bin/bash
# A/B variants of the fused attention block, built HERE (hipcc cross-compiles gfx950) into zonos_vibes_amd/ab/, which
# git ignores but gpurun ships: lib<name>.so (the product library with zmi_attnblk.hip rebuilt with the given -D flags)
# and libstamps_<name>.so (the same with the in-kernel phase stamps, for tools/attnblk_stamps.py).
#   tools/build_ab.sh <name> [-DFLAG=V ...]
# SRC=<file stem> rebuilds another source instead (e.g. SRC=zmi_mambablk).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
SRC=${SRC:-zmi_attnblk}
python -m zonos_vibes_amd.build > /dev/null
mkdir -p zonos_vibes_amd/ab /tmp/ab_$name
CXX="/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc"
$CXX "$@" -c zonos_vibes_amd/csrc/$SRC.hip -o /tmp/ab_$name/p.o &
$CXX "$@" -DZMI_ATTN_STAMPS -DZMI_GEMV_STAMPS -c zonos_vibes_amd/csrc/$SRC.hip -o /tmp/ab_$name/s.o &
wait
others=$(ls zonos_vibes_amd/build/*.o | grep -v "/$SRC\.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others /tmp/ab_$name/p.o -o zonos_vibes_amd/ab/lib$name.so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others /tmp/ab_$name/s.o -o zonos_vibes_amd/ab/libstamps_$name.so
