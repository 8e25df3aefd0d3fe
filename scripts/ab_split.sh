#!/bin/bash
# mixed16: interleaved mixed kernel (0) against the kind split (6) at two LDS budgets; the halves alone
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_split}
mkdir -p "$out"
python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 3:0:256:1,6:0:256:1,7:0:256:1 --norms > "$out/mixed16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config sq16 --rounds 3 --reps 5 --variants 0:0:256:1 --norms > "$out/sq16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config ground16 --rounds 3 --reps 5 --variants 2:0:256:1,5:0:256:1,5:64:256:1,5:80:256:1 --norms > "$out/ground16.jsonl"
