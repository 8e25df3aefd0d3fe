#!/bin/bash
# Round 6: the list tiles capped at four waves per SIMD (127 VGPRs, 2 spilled) against the 129-VGPR build
# (three waves per SIMD), same process, alternating order; variant 6 in both.   scripts/r6_split_probe5.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
L=centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_v6_129.so
timeout -k 10 200 python3 -u scripts/variant_bitwise.py --config mixed16 --batch 20011 --variants 6:0:256:1 > "$out/bitwise.jsonl" || exit $?
timeout -k 10 300 python3 -u scripts/ab_libs.py --config mixed16 --rounds 4 --reps 10 --tuning 6:0:256:1 --libs $L > "$out/mixed16.jsonl" || exit $?
timeout -k 10 200 python3 -u scripts/ab_libs.py --config mixed16 --batch 131072 --rounds 4 --reps 20 --tuning 6:0:256:1 --libs $L > "$out/mixed16_shard.jsonl" || exit $?
timeout -k 10 200 python3 -u scripts/ab_libs.py --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 10 --tuning 6:0:256:1 --libs $L > "$out/list_sq_524k.jsonl" || exit $?
timeout -k 10 200 python3 -u scripts/ab_libs.py --config mixed16 --batch 524288 --tags all_ground --rounds 3 --reps 10 --tuning 6:0:256:1 --libs $L > "$out/list_ground_524k.jsonl" || exit $?
echo done
