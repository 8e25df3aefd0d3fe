#!/bin/bash
# Round 6: IPOPT's Jacobian regularisation in the engine (cpl_kkt_aug_kernel) — the solve-engine GPU
# tests, TestBasic's outcomes with it on the GPU; then the small-batch eval probe.   scripts/r6_jacreg.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -s -m gpu tests/test_gpu_solve_engine.py > "$out/tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u scripts/testbasic_outcomes.py gpu ipopt > "$out/testbasic_gpu_ipopt.jsonl" 2> "$out/testbasic.err" || exit $?
timeout -k 10 300 bash scripts/r6_small_batch_probe.sh "$out/small" || exit $?
echo done
