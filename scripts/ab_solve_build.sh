#!/bin/bash
# A solve-engine change against a previous library build (the round-4 g*.sh sessions, parameterised):
# bitwise solve digests at each batch size and TestBasic's four outcomes for both builds, the solve GPU
# tests on the in-tree build, then the latency / 8 192-solve A/B (scripts/ab_solve.sh).  GPU box.
#   scripts/ab_solve_build.sh OUT LIB_A ["1 64 8192"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}; A=${2:?library A}; batches=${3:-"1 64 8192"}
B=centroidalplanner_amd/libcpl_mi355x.so
mkdir -p "$out"
for b in $batches; do
  CPL_LIB=$A timeout -k 10 120 python -u scripts/solve_digest.py --batch "$b" > "$out/digest_A_B$b.jsonl" || exit $?
  timeout -k 10 120 python -u scripts/solve_digest.py --batch "$b" > "$out/digest_B_B$b.jsonl" || exit $?
done
CPL_LIB=$A timeout -k 10 200 python -u scripts/testbasic_outcomes.py gpu > "$out/testbasic_A.jsonl" || exit $?
timeout -k 10 200 python -u scripts/testbasic_outcomes.py gpu > "$out/testbasic_B.jsonl" || exit $?
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_solve_engine.py \
  tests/test_batch_solve.py tests/test_oracle_pinning.py tests/test_pycpl.py tests/test_ipm_kernels.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
bash scripts/ab_solve.sh "$out/ab_solve" "$A" "$B"
