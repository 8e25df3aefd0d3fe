# round-5 GPU session: Superquadric tiles with the cone items in phase 1 and the values items in phase 2 (cf)
set -o pipefail
O=gpurun_out/r5_g21; mkdir -p $O
bash scripts/ab_eval.sh $O/cf centroidalplanner_amd/libcpl_mi355x.so build/libcpl_cf.so sq8 sq16 || exit $?
