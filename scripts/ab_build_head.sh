#!/bin/bash
# Build libsa_hip.so of a git revision (default HEAD) into ab/<name>/ for an
# interleaved A/B against the working tree (scripts/ab_run.sh <name>)
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}; name=${2:-head}
tmp=$(mktemp -d)
git archive "$rev" hpc_suffix_array_amd/csrc include | tar -x -C "$tmp"
C=$tmp/hpc_suffix_array_amd/csrc
AB=${AB_DIR:-ab}; mkdir -p $AB/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c -x hip $C/sa_build.hip -o $AB/$name/sa_build.o
g++ -O3 -std=c++17 -fPIC -c $C/sa_dropin.cpp -o $AB/$name/sa_dropin.o
g++ -O3 -std=c++17 -fPIC -c $C/sa_debug.cpp -o $AB/$name/sa_debug.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -rdynamic $AB/$name/sa_build.o $AB/$name/sa_dropin.o $AB/$name/sa_debug.o -o $AB/$name/libsa_hip.so
rm -rf "$tmp"
