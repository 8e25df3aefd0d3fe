#!/bin/bash
# Same-box A/B of two library builds on the solve loop: single-instance latency
# (scripts/solve_latency.py) and 8 192 concurrent solves (bench.py --config solve5, both Hessian
# modes), alternating A and B twice.  usage: scripts/ab_solve.sh OUTDIR [LIB_A] [LIB_B]
set -e
out=${1:-gpurun_out/ab_solve}
A=${2:-build/libcpl_old.so}
B=${3:-centroidalplanner_amd/libcpl_mi355x.so}
mkdir -p "$out"
for rep in 1 2; do
  for tag in A B; do
    lib=$A; [ $tag = B ] && lib=$B
    CPL_LIB=$lib timeout -k 10 120 python -u scripts/solve_latency.py --reps 7 > "$out/lat_${tag}_r${rep}.json"
    CPL_LIB=$lib timeout -k 10 120 python -u bench.py --config solve5 --hessian limited-memory --steps 3 --no-cpu --no-pmc \
      > "$out/s5lm_${tag}_r${rep}.json"
    CPL_LIB=$lib timeout -k 10 120 python -u bench.py --config solve5 --hessian exact --steps 3 --no-cpu --no-pmc \
      > "$out/s5ex_${tag}_r${rep}.json"
  done
done
