#!/bin/bash
# VALU counters of the eval kernel for one config (run on the GPU box, each pass its own rocprofv3
# run with its own time limit).  usage: scripts/pmc_valu.sh <config> [batch]
cfg=$1; batch=${2:-0}
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
out="$root/gpurun_out/pmc_valu/$cfg"
mkdir -p "$out"
P1="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU"
P2="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$out/p$i" -o p -- \
    python3 "$root/bench.py" --pmc-child 1 --config "$cfg" --batch "$batch" > "$out/p$i.log" 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o k -- \
  python3 "$root/bench.py" --pmc-child 1 --config "$cfg" --batch "$batch" > "$out/kt.log" 2>&1 || exit $?
