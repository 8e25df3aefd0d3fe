#!/bin/bash
# the dense A entries with 32-bit index divisions: bitwise digests against build/libcpl_fin2.so,
# the solve tests, the solve loop A/B, the solve5 (L-BFGS) kernel profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g34}
mkdir -p "$out"
for B in 64 8192; do
  CPL_LIB=build/libcpl_fin2.so timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_A_B$B.jsonl" || exit $?
  timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_B_B$B.jsonl" || exit $?
done
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_solve_engine.py tests/test_batch_solve.py tests/test_oracle_pinning.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
bash scripts/ab_solve.sh "$out/ab_solve" build/libcpl_fin2.so centroidalplanner_amd/libcpl_mi355x.so || exit $?
