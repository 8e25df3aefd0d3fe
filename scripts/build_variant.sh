#!/bin/bash
# Builds the HIP library from a copy of csrc/ (edited by the caller) into build/<name>.so, for
# scripts/ab_libs.py.  usage: scripts/build_variant.sh <name> <dir with the sources>
name=$1; src=$2
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/build/include"
cp "$root/include/cpl_mi355x.h" "$root/build/include/"
sed -i 's#../../include/cpl_mi355x.h#../include/cpl_mi355x.h#' "$src/cpl_layout.hpp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -std=c++17 -fPIC -shared -w \
  "$src/cpl_host.cpp" "$src/cpl_kernels.hip" "$src/cpl_kkt.hip" "$src/cpl_ipm.hip" "$src/cpl_solver.hip" "$src/cpl_check.hip" -o "$root/build/$name.so"
