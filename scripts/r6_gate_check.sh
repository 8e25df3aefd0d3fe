#!/bin/bash
# Round 6: the small-batch iteration's soft-step evaluation gated on the device (no launch work when no
# instance tries a soft step) — solve digests against the build before (build/libcpl_prevgate.so), the
# single-solve latency of both, the solve-engine GPU tests.   scripts/r6_gate_check.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
for B in 1 64 300; do
  timeout -k 10 200 python -u scripts/solve_digest.py --batch $B > "$out/digest_new_$B.jsonl" 2>> "$out/err.txt" || exit $?
  CPL_LIB=build/libcpl_prevgate.so timeout -k 10 200 python -u scripts/solve_digest.py --batch $B > "$out/digest_prev_$B.jsonl" 2>> "$out/err.txt" || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python -u scripts/solve_latency.py --reps 10 > "$out/latency_new_$r.json" 2>> "$out/err.txt" || exit $?
  CPL_LIB=build/libcpl_prevgate.so timeout -k 10 200 python -u scripts/solve_latency.py --reps 10 > "$out/latency_prev_$r.json" 2>> "$out/err.txt" || exit $?
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_solve_engine.py tests/test_batch_solve.py > "$out/tests.log" 2>&1 || exit $?
echo done
