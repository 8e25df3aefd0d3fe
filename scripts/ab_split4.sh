#!/bin/bash
# mixed16 split modes after the list loaders' changes: concurrent / sequential halves, entry-half LDS
# budget, LDS-staged / Jacobian-direct Superquadric half; the halves alone (one kind through the list)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_split4}
mkdir -p "$out"
python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 0:0:256:1,6:48:256:1,7:0:256:1,7:48:256:1,7:0:256:1:4,7:48:256:1:4,6:0:256:1:4 --norms > "$out/mixed16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_ground --rounds 3 --reps 5 --variants 6:0:256:1,6:48:256:1 --norms > "$out/mixed16_allground.jsonl" || exit $?
python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 5 --variants 6:0:256:1,7:0:256:1 --norms > "$out/mixed16_allsq.jsonl" || exit $?
python -u scripts/ab_kernels.py --config ground16 --rounds 3 --reps 5 --variants 0:0:256:1 --norms > "$out/ground16.jsonl" || exit $?
python -u scripts/ab_kernels.py --config sq16 --rounds 3 --reps 5 --variants 0:0:256:1 --norms > "$out/sq16.jsonl"
