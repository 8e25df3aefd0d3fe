#!/bin/bash
# solve5 (L-BFGS) kernel breakdown, the single solve with and without the HIP graph, the split's LDS budgets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g18}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_s5" -o run -- \
  python3 bench.py --config solve5 --hessian limited-memory --steps 2 --warmup 1 --no-pmc --no-cpu --no-check --no-side > "$out/s5.json" || exit $?
timeout -k 10 120 python -u scripts/solve_latency.py --reps 10 --only limited-memory:1 > "$out/lat_graph.json" || exit $?
timeout -k 10 120 python -u scripts/solve_latency.py --reps 10 --only limited-memory:1 --no-graph > "$out/lat_nograph.json" || exit $?
timeout -k 10 200 python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 7:40:256:1,7:48:256:1,7:56:256:1,7:64:256:1 --norms > "$out/mixed16_lds.jsonl" || exit $?
for B in 1 8192; do
  timeout -k 10 60 build/kkt_probe_prev $B > "$out/kkt_prev_B$B.txt" || exit $?
  timeout -k 10 60 scripts/kkt_probe $B > "$out/kkt_new_B$B.txt" || exit $?
done
bash scripts/ab_solve.sh "$out/ab_solve" build/libcpl_prev.so centroidalplanner_amd/libcpl_mi355x.so
