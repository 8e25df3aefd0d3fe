# round-5 GPU session: Superquadric scratch strides chosen by the LDS bank model (bank) — A/B against the in-tree build
set -o pipefail
O=gpurun_out/r5_g26; mkdir -p $O
bash scripts/ab_eval.sh $O/bank centroidalplanner_amd/libcpl_mi355x.so build/libcpl_bank.so sq8 sq16 || exit $?
