# round-5 GPU session: the statics values item's contacts loaded four at a time (stv) — A/B against the in-tree build
set -o pipefail
O=gpurun_out/r5_g20; mkdir -p $O
bash scripts/ab_eval.sh $O/stv centroidalplanner_amd/libcpl_mi355x.so build/libcpl_stv.so sq16 sq8 ground4_1m mixed16 || exit $?
