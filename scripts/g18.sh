#!/bin/bash
# the pipelined small-batch iteration (head / tail graphs) and the DPP change: solve tests, KKT probe
# hashes and cycles, single-solve latency of three builds, solve5 (L-BFGS) kernel breakdown, the
# split's LDS budgets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g18}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_solve_engine.py tests/test_batch_solve.py tests/test_pycpl.py tests/test_oracle_pinning.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
for B in 1 8192; do
  timeout -k 10 60 build/kkt_probe_prev $B > "$out/kkt_prev_B$B.txt" || exit $?
  timeout -k 10 60 scripts/kkt_probe $B > "$out/kkt_new_B$B.txt" || exit $?
done
for rep in 1 2; do
  for lib in build/libcpl_prev.so build/libcpl_dpp.so centroidalplanner_amd/libcpl_mi355x.so; do
    tag=$(basename $lib .so)
    CPL_LIB=$lib timeout -k 10 120 python -u scripts/solve_latency.py --reps 10 > "$out/lat_${tag}_r$rep.json" || exit $?
  done
  for lib in build/libcpl_prev.so centroidalplanner_amd/libcpl_mi355x.so; do
    tag=$(basename $lib .so)
    CPL_LIB=$lib timeout -k 10 120 python -u bench.py --config solve5 --hessian limited-memory --steps 3 --no-cpu --no-pmc > "$out/s5lm_${tag}_r$rep.json" || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_s5" -o run -- \
  python3 bench.py --config solve5 --hessian limited-memory --steps 2 --warmup 1 --no-pmc --no-cpu --no-check --no-side > "$out/s5.json" || exit $?
timeout -k 10 200 python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 7:40:256:1,7:48:256:1,7:56:256:1,7:64:256:1 --norms > "$out/mixed16_lds.jsonl"
