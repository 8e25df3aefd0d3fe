#!/bin/bash
# the single-instance speculative next iteration: bitwise digests at B = 1 / 64 and TestBasic's outcomes
# against build/libcpl_cap.so, the solve tests, the single-solve latency A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g29}
mkdir -p "$out"
for B in 1 64; do
  CPL_LIB=build/libcpl_cap.so timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_A_B$B.jsonl" || exit $?
  timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_B_B$B.jsonl" || exit $?
done
CPL_LIB=build/libcpl_cap.so timeout -k 10 200 python -u scripts/testbasic_outcomes.py gpu > "$out/testbasic_A.jsonl" || exit $?
timeout -k 10 200 python -u scripts/testbasic_outcomes.py gpu > "$out/testbasic_B.jsonl" || exit $?
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_solve_engine.py tests/test_batch_solve.py tests/test_oracle_pinning.py tests/test_pycpl.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
for rep in 1 2; do
  for tag in A B; do
    lib=build/libcpl_cap.so; [ $tag = B ] && lib=centroidalplanner_amd/libcpl_mi355x.so
    CPL_LIB=$lib timeout -k 10 120 python -u scripts/solve_latency.py --reps 10 > "$out/lat_${tag}_r$rep.json" || exit $?
  done
done
