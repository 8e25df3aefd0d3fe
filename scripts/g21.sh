#!/bin/bash
# the register M build of the limited-memory Newton setup: bitwise digests against build/libcpl_lbw.so,
# the solve tests, the solve loop A/B, the solve5 (L-BFGS) kernel profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g21}
mkdir -p "$out"
for B in 64 8192; do
  CPL_LIB=build/libcpl_lbw.so timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_A_B$B.jsonl" || exit $?
  timeout -k 10 120 python -u scripts/solve_digest.py --batch $B > "$out/digest_B_B$B.jsonl" || exit $?
done
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_solve_engine.py tests/test_batch_solve.py tests/test_oracle_pinning.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
bash scripts/ab_solve.sh "$out/ab_solve" build/libcpl_lbw.so centroidalplanner_amd/libcpl_mi355x.so || exit $?
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_s5" -o run -- \
  python3 bench.py --config solve5 --hessian limited-memory --steps 2 --warmup 1 --no-pmc --no-cpu --no-check --no-side > "$out/s5.json"
CPL_LIB=build/libcpl_ls3.so timeout -k 10 120 python -u scripts/solve_digest.py --batch 8192 > "$out/digest_C_B8192.jsonl" || exit $?
bash scripts/ab_solve.sh "$out/ab_ls3" centroidalplanner_amd/libcpl_mi355x.so build/libcpl_ls3.so
