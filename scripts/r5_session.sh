# round-5 GPU session: the statics sums as chain items in Superquadric tiles (chain) — A/B against the in-tree build
set -o pipefail
O=gpurun_out/r5_g22; mkdir -p $O
bash scripts/ab_eval.sh $O/chain centroidalplanner_amd/libcpl_mi355x.so build/libcpl_chain.so sq16 sq8 || exit $?
