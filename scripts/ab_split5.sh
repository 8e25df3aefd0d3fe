#!/bin/bash
# the kind split's Superquadric list launch: a persistent grid walking the list's tiles (the in-tree
# build) against one tile per workgroup over every possible tile (build/libcpl_noloop.so), Jacobian-
# direct half and 48 KiB budgets; then the in-tree default (variant 0) against the forced variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_split5}
mkdir -p "$out"
L=centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_noloop.so
python -u scripts/ab_libs.py --config mixed16 --rounds 3 --reps 5 --tuning 7:48:256:1 --libs $L > "$out/mixed16_7_48.jsonl" || exit $?
python -u scripts/ab_libs.py --config mixed16 --batch 524288 --tags all_ground --rounds 3 --reps 5 --tuning 7:48:256:1 --libs $L > "$out/allground_7_48.jsonl" || exit $?
python -u scripts/ab_libs.py --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 5 --tuning 7:48:256:1 --libs $L > "$out/allsq_7_48.jsonl" || exit $?
python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 0:0:256:1,7:48:256:1,6:48:256:1,3:0:256:1 --norms > "$out/mixed16_default.jsonl"
