#!/bin/bash
# End-of-round evidence on one gpurun box: GPU test suite, smoke, the default bench line, the bench
# under rocprofv3 (kernel trace + stats, CSV) with the per-grid breakdown of the trace
# (scripts/trace_by_grid.py: the headline kernel's average over its own grid, recomputable from the
# committed CSV), the side configs' own lines, the single-solve latency and TestBasic's scenarios on the
# GPU.  Each GPU step has its own time limit; a fault, abort or time-out (exit status >= 124) ends the
# script there (test failures do not).  usage: scripts/final_evidence.sh OUTDIR [PART]
# (PART 1: tests, smoke, the default bench line and its profile; 2: the side configs, the latency and
# TestBasic; default both)
out=${1:-gpurun_out/final}
part=${2:-all}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # step <seconds> <command...>
  local secs=$1
  shift
  echo "=== [$(date +%T)] $*"
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "=== rc=$rc"
  if [ "$rc" -ge 124 ]; then
    echo "stopping: fault/abort/timeout"
    exit "$rc"
  fi
  return 0
}
if [ "$part" != 2 ]; then
step 900 bash -c "python -u -m pytest -q --timeout 240 --timeout-method thread tests -m gpu > $out/gpu_tests.log 2>&1"
step 300 bash -c "python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > $out/smoke.log 2>&1"
step 300 bash -c "python -u bench.py > $out/bench_default.json 2> $out/bench_default.err"
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
  python3 bench.py --steps 20 --no-pmc --no-cpu --no-check --no-side
trace=$(find "$out/prof" -name "*kernel_trace.csv" | head -1)
stats=$(find "$out/prof" -name "*kernel_stats.csv" | head -1)
[ -n "$trace" ] && python scripts/trace_by_grid.py "$trace" "$out/kernel_by_grid_bench_default.csv" > "$out/kernel_by_grid_top.txt"
[ -n "$stats" ] && cp "$stats" "$out/kernel_stats_bench_default.csv"
fi
[ "$part" = 1 ] && { echo done; exit 0; }
step 300 bash -c "python -u bench.py --config sq8 > $out/bench_sq8.json 2> $out/bench_sq8.err"
step 300 bash -c "python -u bench.py --config mixed16 > $out/bench_mixed16.json 2> $out/bench_mixed16.err"
step 300 bash -c "python -u bench.py --config solve5 --hessian limited-memory > $out/bench_solve5_lbfgs.json 2> $out/bench_solve5_lbfgs.err"
step 300 bash -c "python -u bench.py --config solve5 > $out/bench_solve5_exact.json 2> $out/bench_solve5_exact.err"
step 300 bash -c "python -u scripts/solve_latency.py --reps 10 > $out/solve_latency.json 2> $out/solve_latency.err"
step 300 bash -c "python -u scripts/testbasic_outcomes.py gpu > $out/testbasic_gpu.jsonl 2> $out/testbasic_gpu.err"
step 300 bash -c "python -u scripts/testbasic_outcomes.py gpu ipopt > $out/testbasic_gpu_ipopt.jsonl 2> $out/testbasic_gpu_ipopt.err"
echo done
