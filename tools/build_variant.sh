#!/bin/bash
# A/B library variant: the whole library rebuilt with extra -D flags into zonos_vibes_amd/var/lib<name>.so
#   tools/build_variant.sh lntasks -DZMI_LN_TASKS
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p zonos_vibes_amd/var /tmp/var_$name
objs=""
for src in zonos_vibes_amd/csrc/*.hip; do
  o=/tmp/var_$name/$(basename $src .hip).o
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izonos_vibes_amd/csrc "$@" \
    -c $src -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o zonos_vibes_amd/var/lib$name.so
echo zonos_vibes_amd/var/lib$name.so
