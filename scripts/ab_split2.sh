#!/bin/bash
# mixed16: the kind split's halves concurrent (side stream) vs one after the other (ablate 4), entry-half
# LDS budgets, Jacobian-direct Superquadric half; sq16 contiguous and ground16 entry alone for reference
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_split2}
mkdir -p "$out"
python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 0:0:256:1,6:0:256:1:4,6:48:256:1,6:48:256:1:4,7:0:256:1:4,3:0:256:1 --norms > "$out/mixed16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config sq16 --rounds 3 --reps 5 --variants 0:0:256:1,0:64:256:1 --norms > "$out/sq16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config ground16 --rounds 3 --reps 5 --variants 0:0:256:1,5:48:256:1 --norms > "$out/ground16.jsonl"
