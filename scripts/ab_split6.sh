#!/bin/bash
# the kind split's launch order (ablation 8: the Ground half issued first) against the default order,
# on the 50/50 mixed batch and on an all-Ground / all-Superquadric mixed-kind batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_split6}
mkdir -p "$out"
V=0:0:256:1,7:48:256:1,7:48:256:1:8,7:48:256:1:4
python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants $V --norms > "$out/mixed16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_ground --rounds 3 --reps 5 --variants $V --norms > "$out/allground.jsonl" || exit $?
python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 5 --variants $V --norms > "$out/allsq.jsonl"
