#!/bin/bash
# Round 6: the regularised systems' corrections inside the fused search (AUGR) — the solve-engine GPU
# tests, the cost against the pivot form, TestBasic with it on.   scripts/r6_jacreg2.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_solve_engine.py > "$out/tests.log" 2>&1 || exit $?
timeout -k 10 500 python -u scripts/jacreg_cost.py > "$out/cost.jsonl" 2> "$out/cost.err" || exit $?
timeout -k 10 300 python -u scripts/testbasic_outcomes.py gpu ipopt > "$out/testbasic_gpu_ipopt.jsonl" 2> "$out/testbasic.err" || exit $?
echo done
