#!/bin/bash
# the partition's scan folded into the write kernel: same-process A/B against the previous build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g26}
mkdir -p "$out"
L=centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_head.so
timeout -k 10 300 python -u scripts/ab_libs.py --config mixed16 --rounds 5 --reps 5 --libs $L > "$out/mixed16.jsonl" || exit $?
timeout -k 10 300 python -u scripts/ab_libs.py --config mixed16 --batch 65536 --rounds 5 --reps 5 --libs $L > "$out/mixed16_64k.jsonl"
