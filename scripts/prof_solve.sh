#!/bin/bash
# The solve loop under rocprofv3 (kernel trace + stats): 8 192 limited-memory solves and the single
# solve (B = 1).  GPU box.  scripts/prof_solve.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_s5" -o run -- \
  python3 bench.py --config solve5 --hessian limited-memory --steps 2 --warmup 1 --no-pmc --no-cpu --no-check --no-side \
  > "$out/s5.json" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_b1" -o run -- \
  python3 scripts/solve_latency.py --reps 5 --only limited-memory:1 > "$out/b1.json"
