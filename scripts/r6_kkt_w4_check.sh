#!/bin/bash
# Round 6: the four-wave KKT form (Z and c_p on four waves at small batches) — the probe against the
# one-wave form, the solve-engine GPU tests, the single-solve latency.   scripts/r6_kkt_w4_check.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
for B in 1 64 256; do
  timeout -k 10 60 ./build/kprobe_base $B > "$out/base_$B.txt" || exit $?
  CPL_KKT_W4=1 timeout -k 10 60 ./build/kprobe_w4 $B > "$out/w4_$B.txt" || exit $?
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_solve_engine.py tests/test_batch_solve.py > "$out/tests.log" 2>&1 || exit $?
timeout -k 10 200 python -u scripts/solve_latency.py --reps 10 > "$out/latency_w4.json" 2> "$out/latency.err" || exit $?
CPL_KKT_W4=0 timeout -k 10 200 python -u scripts/solve_latency.py --reps 10 > "$out/latency_w1.json" 2>> "$out/latency.err" || exit $?
echo done
