#!/bin/bash
# Round 6: one B = 1 L-BFGS solve under the kernel trace (per-iteration kernel durations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_b1" -o run -- \
  python3 scripts/solve_latency.py --reps 3 --only limited-memory:1 > "$out/b1.json"
