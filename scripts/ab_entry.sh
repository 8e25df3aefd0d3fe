#!/bin/bash
# A/B of the entry-parallel kernel (variant 5) against the pipelined one (2) in one process per config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_entry}
mkdir -p "$out"
for cfg in ground4_1m ground16 ground4; do
  python -u scripts/ab_kernels.py --config $cfg --rounds 5 --reps 20 --variants 2:0:256:1,5:0:256:1,5:64:256:1,5:32:256:1 --norms > "$out/$cfg.jsonl" || exit $?
done
python -u scripts/ab_kernels.py --config ground4_1m --rounds 3 --reps 20 --variants 2:0:256:1,5:0:256:1 --outputs g,jac,f,grad > "$out/ground4_1m_fgrad.jsonl"
python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 0:0:256:1,6:0:256:1 --norms > "$out/mixed16.jsonl"
