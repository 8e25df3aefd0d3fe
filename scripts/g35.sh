#!/bin/bash
# the post-step quantities in the fused search kernel's prologue (below LS_GF_MIN): bitwise digests at
# B = 1 / 64 / 8 192 and TestBasic's outcomes against build/libcpl_fin3.so, the solve tests, the solve A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g35}
mkdir -p "$out"
A=build/libcpl_fin3.so
for B in 1 64 8192; do
  CPL_LIB=$A timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_A_B$B.jsonl" || exit $?
  timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_B_B$B.jsonl" || exit $?
done
CPL_LIB=$A timeout -k 10 200 python -u scripts/testbasic_outcomes.py gpu > "$out/testbasic_A.jsonl" || exit $?
timeout -k 10 200 python -u scripts/testbasic_outcomes.py gpu > "$out/testbasic_B.jsonl" || exit $?
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_solve_engine.py tests/test_batch_solve.py tests/test_oracle_pinning.py tests/test_pycpl.py tests/test_ipm_kernels.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
bash scripts/ab_solve.sh "$out/ab_solve" $A centroidalplanner_amd/libcpl_mi355x.so
