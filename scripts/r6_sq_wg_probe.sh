#!/bin/bash
# Round 6: configs[2] (262 144 x 8 Superquadric) tile kernel on 128-thread workgroups (two waves, half the
# tile: twice the workgroups per CU at the same waves per SIMD) against the default 256.
# scripts/r6_sq_wg_probe.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
AB="python3 -u scripts/ab_kernels.py"
V="0:0:256:1,3:0:128:1,3:16:128:1,3:20:128:1,3:24:128:1,3:32:128:1,3:0:256:1"
timeout -k 10 400 $AB --config sq8 --rounds 5 --reps 20 --variants $V --norms > "$out/sq8.jsonl" || exit $?
timeout -k 10 400 $AB --config sq8 --batch 524288 --rounds 3 --reps 10 --variants $V --norms > "$out/sq8_524k.jsonl" || exit $?
echo done
