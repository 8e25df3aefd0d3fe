#!/bin/bash
# HBM traffic of one eval config per kernel (FETCH_SIZE and WRITE_SIZE in separate --pmc passes: the
# two do not fit one pass's TCC slots), summarised per kernel by scripts/pmc_summary.py.  GPU box.
#   scripts/pmc_traffic.sh CONFIG OUT [ab_kernels variant, default 0:0:256:1] [extra ab_kernels args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cfg=${1:?config}; out=${2:?out dir}; var=${3:-0:0:256:1}; shift 3 2>/dev/null
mkdir -p "$out"
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/$ctr" -o p -- \
    python3 scripts/ab_kernels.py --config "$cfg" --rounds 1 --reps 2 --variants "$var" "$@" > "$out/$ctr.log" 2>&1 || exit $?
done
for k in tile_kernel entry_kernel kind_ residual; do
  echo "== $k"; python3 scripts/pmc_summary.py "$out" "$k"
done > "$out/summary.txt"
