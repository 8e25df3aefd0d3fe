#!/bin/bash
# sq8 tile kernel instruction / LDS / wait counters (separate --pmc passes, each under its own limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/g24
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # run <tag> <counters...>
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$tag" -o p -- \
    python3 scripts/ab_kernels.py --config sq8 --rounds 1 --reps 3 --variants 0:0:256:1 > "$out/$tag.log" 2>&1
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS || exit $?
run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY || exit $?
run c SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA
