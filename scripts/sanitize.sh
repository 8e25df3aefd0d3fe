#!/bin/bash
# Host-side sanitizer builds (SURVEY.md section 5 "Race detection / sanitizers"): AddressSanitizer +
# UndefinedBehaviorSanitizer on the host code with raw indexing — the oracle (oracle/cpl_oracle.c,
# oracle/cpl_solve_host.c), the C++ facade (libcpl_host.so) and its test driver (tests/cpp/test_host.cpp)
# — then the CPU test suite and the C++ CPU cases under them.  CPU only (no GPU code is instrumented:
# the facade is host C++, built -x c++ with -fno-gpu-sanitize).  Usage: scripts/sanitize.sh [pytest args]
set -euo pipefail
root=$(cd "$(dirname "$0")/.." && pwd)
out="$root/tests/_build/asan"
mkdir -p "$out"
san="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"

# 1. the oracle (gcc): same flags as oracle/Makefile plus the sanitizers
gcc -ffp-contract=off -fno-fast-math -fPIC -fopenmp -Wall -Wextra -std=c11 $san -shared \
  -o "$out/libcpl_oracle_asan.so" "$root/oracle/cpl_oracle.c" "$root/oracle/cpl_solve_host.c" -lm

# 2. the C++ facade and the C++ test driver (clang through hipcc, host code only)
rocm=${ROCM_PATH:-/opt/rocm}
pkg="$root/centroidalplanner_amd"
/opt/rocm/bin/hipcc -x c++ -fno-gpu-sanitize $san -std=c++17 -fPIC -shared -Wall -D__HIP_PLATFORM_AMD__ \
  -I"$root/include" -I"$rocm/include" "$pkg"/host/cpl_problem.cpp "$pkg"/host/cpl_planner.cpp \
  "$pkg"/host/cpl_broker.cpp "$pkg"/host/cpl_native.cpp -o "$out/libcpl_host.so" \
  -L"$pkg" -lcpl_mi355x -L"$rocm/lib" -lamdhip64 -Wl,-rpath,"$pkg"
/opt/rocm/bin/hipcc -x c++ -fno-gpu-sanitize $san -std=c++17 -Wall -D__HIP_PLATFORM_AMD__ \
  -I"$root/include" -I"$rocm/include" "$root/tests/cpp/test_host.cpp" -o "$out/test_host" \
  -L"$out" -lcpl_host -L"$pkg" -lcpl_mi355x -L"$rocm/lib" -lamdhip64 -ldl -Wl,-rpath,"$out" -Wl,-rpath,"$pkg"

# the HIP runtime allocates for the life of the process: leak reports off, every error fatal
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1

echo "== C++ facade CPU cases under ASan/UBSan"
"$out/test_host" | tail -3

echo "== CPU test suite with the sanitized oracle (LD_PRELOAD: the interpreter itself is not instrumented)"
cd "$root"
CPL_ORACLE_LIB="$out/libcpl_oracle_asan.so" LD_PRELOAD="$(gcc -print-file-name=libasan.so)" \
  python -m pytest tests/ -x -q -m "not gpu" -p no:cacheprovider "$@"
