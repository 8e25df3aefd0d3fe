#!/bin/bash
# sq8 / sq16 / mixed16 eval kernels: the current library against build/libcpl_old.so (same process), and
# the Superquadric tile variants (LDS staging vs Jacobian rows written directly, LDS budgets)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_sq_tiles}
mkdir -p "$out"
for cfg in sq8 sq16 mixed16; do
  python -u scripts/ab_libs.py --config $cfg --rounds 3 --reps 10 --libs centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_old.so > "$out/libs_$cfg.jsonl" || exit $?
done
python -u scripts/ab_kernels.py --config sq8 --rounds 3 --reps 10 --variants 0:0:256:1,4:0:256:1,0:40:256:1,4:32:256:1,4:40:256:1,0:64:256:1 --norms > "$out/var_sq8.jsonl" || exit $?
python -u scripts/ab_kernels.py --config mixed16 --rounds 3 --reps 5 --variants 0:0:256:1,6:0:256:1,3:0:256:1 --norms > "$out/var_mixed16.jsonl"
