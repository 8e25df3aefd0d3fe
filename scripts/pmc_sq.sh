#!/bin/bash
# PMC pass over the eval kernels of one config (run on the GPU box).  usage: pmc_sq.sh <config> <out> <counters...>
cfg=$1; out=$2; shift 2
cd /tmp && export TMPDIR=/tmp
exec_rocprof() { rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$out" -o p -- python3 "$GRAFT_REPO_ROOT/scripts/ab_kernels.py" --config "$cfg" --rounds 1 --reps 3 --variants 0:32:256:1:0; }
exec_rocprof "$@"
