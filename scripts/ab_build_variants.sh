#!/bin/bash
# Build libsa_hip.so variants for A/B timing into ab/<name>/libsa_hip.so; run
# them with scripts/ab_run.sh (SA_LIB_PATH points bench.py at one).  A
# variant name is a list of -D overrides joined by '+', e.g.
#   SA_ITEMS_B=10+SA_BS_GRID=512
set -e
cd "$(dirname "$0")/.."
C=hpc_suffix_array_amd/csrc
make -s -C $C
for v in "$@"; do
  AB=${AB_DIR:-ab}; mkdir -p $AB/$v
  defs=$(echo "$v" | tr '+' '\n' | sed 's/^/-D/' | tr '\n' ' ')
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $defs -c -x hip $C/sa_build.hip -o $AB/$v/sa_build.o &
done
wait
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -rdynamic $AB/$v/sa_build.o $C/build/sa_dropin.o $C/build/sa_debug.o -o $AB/$v/libsa_hip.so
done
