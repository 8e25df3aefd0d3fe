#!/bin/bash
# Round 6: the split's remaining costs — the empty Superquadric workgroups past the list (ablate 16384:
# the grid for half the batch, valid for the alternating tags), the halves back to back (4 | 256) and the
# Ground half issued first (8).   scripts/r6_split_probe7.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
AB="python3 -u scripts/ab_kernels.py"
V="0:0:256:1,0:0:256:1:16384,0:0:256:1:260,0:0:256:1:8"
# (16384 is bitwise on random and all-Ground tags, not all-Superquadric: a pricing probe only)
timeout -k 10 400 $AB --config mixed16 --rounds 4 --reps 10 --variants $V > "$out/mixed16.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 131072 --rounds 4 --reps 20 --variants $V > "$out/mixed16_shard.jsonl" || exit $?
echo done
