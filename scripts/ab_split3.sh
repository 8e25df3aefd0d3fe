#!/bin/bash
# the kind split's Superquadric half alone (every instance Superquadric, through the list launch) against
# the contiguous Superquadric kernel on the same points, and the Ground half alone against the entry
# kernel's contiguous launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_split3}
mkdir -p "$out"
python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 5 --variants 6:0:256:1,7:0:256:1,3:0:256:1 --norms > "$out/mixed16_allsq.jsonl" || exit $?
python -u scripts/ab_kernels.py --config sq16 --rounds 3 --reps 5 --variants 0:0:256:1 --norms > "$out/sq16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_ground --rounds 3 --reps 5 --variants 6:0:256:1,6:48:256:1,3:0:256:1 --norms > "$out/mixed16_allground.jsonl" || exit $?
python -u scripts/ab_kernels.py --config ground16 --rounds 3 --reps 5 --variants 5:0:256:1,5:48:256:1 --norms > "$out/ground16.jsonl"
