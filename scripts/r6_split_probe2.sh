#!/bin/bash
# Round 6: the mixed kind split with the Superquadric half on LDS-staged uniform-axis list tiles
# (variant 6) and the Ground half's compute waves at a raised priority (ablate 1024 / 2048), against the
# default; bitwise checks first.   scripts/r6_split_probe2.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
AB="python3 -u scripts/ab_kernels.py"
V="0:0:256:1,6:0:256:1,6:0:256:1:1024,6:0:256:1:2048,0:0:256:1:1024"
timeout -k 10 200 python3 -u scripts/variant_bitwise.py --config mixed16 --batch 20011 --variants 6:0:256:1,6:0:256:1:1024,0:0:256:1:1024 > "$out/bitwise.jsonl" || exit $?
timeout -k 10 400 $AB --config mixed16 --rounds 4 --reps 10 --variants $V > "$out/mixed16.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 131072 --rounds 4 --reps 20 --variants $V > "$out/mixed16_shard.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 10 --variants 0:0:256:1,6:0:256:1 > "$out/list_sq_524k.jsonl" || exit $?
echo done
