#!/bin/bash
# Round 6: the solve engine against a baseline build — the new solve tests, bitwise digests at
# B = 1 / 64 / 8 192 for both builds, then scripts/ab_solve.sh (latency + solve5, alternating).
#   scripts/r6_solve_ab.sh OUT BASELINE_LIB
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out}; A=${2:?baseline}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_batch_solve.py -m gpu -x -q --timeout 240 --timeout-method thread -k "compaction or tail" > "$out/tests.log" 2>&1 || exit $?
for b in 1 64 8192; do
  CPL_LIB=$A timeout -k 10 120 python -u scripts/solve_digest.py --batch $b > "$out/digest_A_B$b.jsonl" || exit $?
  timeout -k 10 120 python -u scripts/solve_digest.py --batch $b > "$out/digest_B_B$b.jsonl" || exit $?
done
bash scripts/ab_solve.sh "$out" "$A" centroidalplanner_amd/libcpl_mi355x.so || exit $?
echo done
