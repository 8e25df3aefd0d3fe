#!/bin/bash
# Round 6: configs[1] (65 536 x 4 Ground) — the pipelined kernel's tile size for small batches (LDS budget
# 24 KiB: T = 8 instances, against the default 48 KiB: T = 16; the grid is the resident workgroups, so the
# last round of tiles leaves part of the GPU idle), and the entry kernel.   scripts/r6_small_batch_probe.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
AB="python3 -u scripts/ab_kernels.py"
V="0:0:256:1,2:24:256:1,5:0:256:1"
timeout -k 10 300 $AB --config ground4 --rounds 5 --reps 50 --variants $V --norms > "$out/ground4_65k.jsonl" || exit $?
timeout -k 10 300 $AB --config ground4 --batch 262144 --rounds 5 --reps 20 --variants $V --norms > "$out/ground4_262k.jsonl" || exit $?
timeout -k 10 300 $AB --config ground4_1m --rounds 3 --reps 10 --variants $V --norms > "$out/ground4_1m.jsonl" || exit $?
echo done
