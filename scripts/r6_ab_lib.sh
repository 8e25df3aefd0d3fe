#!/bin/bash
# Round 6: the current library against build/<B>.so on the mixed configs (same process, alternating order),
# bitwise checks of the default variant.   scripts/r6_ab_lib.sh OUT B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}; B=${2:?baseline library}
mkdir -p "$out"
L=centroidalplanner_amd/libcpl_mi355x.so,$B
timeout -k 10 200 python3 -u scripts/variant_bitwise.py --config mixed16 --batch 20011 --variants 7:0:256:1 > "$out/bitwise.jsonl" || exit $?
timeout -k 10 300 python3 -u scripts/ab_libs.py --config mixed16 --rounds 4 --reps 10 --libs $L > "$out/mixed16.jsonl" || exit $?
timeout -k 10 200 python3 -u scripts/ab_libs.py --config mixed16 --batch 131072 --rounds 4 --reps 20 --libs $L > "$out/mixed16_shard.jsonl" || exit $?
timeout -k 10 200 python3 -u scripts/ab_libs.py --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 10 --libs $L > "$out/list_sq_524k.jsonl" || exit $?
timeout -k 10 200 python3 -u scripts/ab_libs.py --config sq16 --rounds 3 --reps 10 --libs $L > "$out/sq16.jsonl" || exit $?
echo done
