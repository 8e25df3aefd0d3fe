#!/bin/bash
# sq8 tile workgroup size (128 / 256 threads) and LDS budgets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g30}
mkdir -p "$out"
timeout -k 10 300 python -u scripts/ab_kernels.py --config sq8 --rounds 4 --reps 5 --variants 0:0:256:1,0:40:256:1,0:44:256:1,0:36:256:1 --norms > "$out/sq8_wg.jsonl"
