#!/bin/bash
# Instruction / LDS / wait counters of one eval config's kernels: three separate --pmc passes (each
# within the per-block slot limits, each under its own time limit).  GPU box.
#   scripts/pmc_eval.sh CONFIG OUT [ab_kernels variant, default 0:0:256:1]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
cfg=${1:?config}; out=${2:?out dir}; var=${3:-0:0:256:1}
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # run <tag> <counters...>
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$tag" -o p -- \
    python3 scripts/ab_kernels.py --config "$cfg" --rounds 1 --reps 3 --variants "$var" > "$out/$tag.log" 2>&1
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_LDS || exit $?
run b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY || exit $?
run c SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA
