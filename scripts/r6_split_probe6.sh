#!/bin/bash
# Round 6: the new split default (LDS-staged uniform-axis list tiles, four waves per SIMD) with the Ground
# walker cap variants (256 = none, 512 = two per CU) and the Ground compute-wave priority (1024).
#   scripts/r6_split_probe6.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
AB="python3 -u scripts/ab_kernels.py"
V="0:0:256:1,0:0:256:1:256,0:0:256:1:512,0:0:256:1:1024,7:0:256:1"
timeout -k 10 200 python3 -u scripts/variant_bitwise.py --config mixed16 --batch 20011 --variants 7:0:256:1,0:0:256:1:256 > "$out/bitwise.jsonl" || exit $?
timeout -k 10 400 $AB --config mixed16 --rounds 4 --reps 10 --variants $V > "$out/mixed16.jsonl" || exit $?
timeout -k 10 300 $AB --config mixed16 --batch 262144 --rounds 4 --reps 20 --variants $V > "$out/mixed16_262k.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 131072 --rounds 4 --reps 20 --variants $V > "$out/mixed16_shard.jsonl" || exit $?
cd /tmp || exit 1
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/kt" -o k -- \
  python3 "$R/scripts/ab_kernels.py" --config mixed16 --rounds 1 --reps 3 --variants 0:0:256:1 > "$R/$out/kt.log" 2>&1 || exit $?
echo done
