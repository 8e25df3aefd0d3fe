#!/bin/bash
# the one-wave KKT kernel's smaller LDS image (packed L, two vector slots): probe hashes and cycles
# against the previous build, the KKT / solve GPU tests, the solve loop against build/libcpl_dpp.so,
# the split's LDS budgets for the mixed batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g19}
mkdir -p "$out"
for B in 1 8192; do
  timeout -k 10 60 build/kkt_probe_prev $B > "$out/kkt_prev_B$B.txt" || exit $?
  timeout -k 10 60 scripts/kkt_probe $B > "$out/kkt_new_B$B.txt" || exit $?
done
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_kkt.py tests/test_ipm_kernels.py tests/test_gpu_solve_engine.py tests/test_batch_solve.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
bash scripts/ab_solve.sh "$out/ab_solve" build/libcpl_dpp.so centroidalplanner_amd/libcpl_mi355x.so || exit $?
timeout -k 10 200 python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 7:0:256:1,7:0:256:1:16,7:0:256:1:32,7:0:256:1:48,7:40:256:1,7:36:256:1,7:32:256:1 --norms > "$out/mixed16_lds.jsonl"
