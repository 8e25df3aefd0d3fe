#!/bin/bash
# the kind split's Ground half on one workgroup per CU (ablation 256), issued first (8) or not
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g27}
mkdir -p "$out"
timeout -k 10 300 python -u scripts/ab_kernels.py --config mixed16 --rounds 4 --reps 5 --variants 0:0:256:1,0:0:256:1:256,0:0:256:1:512,0:0:256:1:288,0:0:256:1:272,0:0:256:1:264 --norms > "$out/mixed16_ground_grid.jsonl"
