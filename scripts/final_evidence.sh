#!/bin/bash
# End-of-round evidence on one gpurun box: GPU test suite, smoke, the default bench line, the bench
# under rocprofv3 (kernel trace + stats, CSV) with the per-grid breakdown of the trace
# (scripts/trace_by_grid.py: the headline kernel's average over its own grid, recomputable from the
# committed CSV), the side configs' own lines and the single-solve latency.  Each GPU step has its
# own time limit; the script stops at the first failure.  usage: scripts/final_evidence.sh OUTDIR
set -e
out=${1:-gpurun_out/final}
mkdir -p "$out"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 240 --timeout-method thread tests -m gpu > "$out/gpu_tests.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
  python3 bench.py --steps 20 --no-pmc --no-cpu --no-check --no-side > "$out/bench_under_rocprof.json" 2> "$out/rocprof.err"
trace=$(find "$out/prof" -name "*kernel_trace.csv" | head -1)
stats=$(find "$out/prof" -name "*kernel_stats.csv" | head -1)
python scripts/trace_by_grid.py "$trace" "$out/kernel_by_grid_bench_default.csv" > "$out/kernel_by_grid_top.txt"
cp "$stats" "$out/kernel_stats_bench_default.csv"
timeout -k 10 300 python -u bench.py --config sq8 > "$out/bench_sq8.json" 2> "$out/bench_sq8.err"
timeout -k 10 300 python -u bench.py --config mixed16 > "$out/bench_mixed16.json" 2> "$out/bench_mixed16.err"
timeout -k 10 300 python -u scripts/solve_latency.py --reps 10 > "$out/solve_latency.json" 2> "$out/solve_latency.err"
timeout -k 10 300 python -u scripts/testbasic_outcomes.py gpu > "$out/testbasic_gpu.jsonl" 2> "$out/testbasic_gpu.err"
echo done
