#!/bin/bash
# same-process A/B of the current library against build/libcpl_old.so on the Superquadric configs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/ab_sq}
mkdir -p "$out"
for cfg in sq8 sq16; do
  python -u scripts/ab_libs.py --config $cfg --rounds 5 --reps 10 --libs centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_old.so > "$out/$cfg.jsonl" || exit $?
done
python -u scripts/ab_libs.py --config mixed16 --rounds 3 --reps 5 --tuning 7:0:256:1 --libs centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_old.so > "$out/mixed16_split_jd.jsonl"
