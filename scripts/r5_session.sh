# round-5 GPU session: the M products of the second-order-correction re-solves with unconditional loads
# (mfma_matvec_g) against the build before
set -o pipefail
O=gpurun_out/r5_g32; mkdir -p $O/ab

for B in 1 64 8192; do
  for t in A B; do
    lib=build/libcpl_pre_kkt.so; [ $t = B ] && lib=centroidalplanner_amd/libcpl_mi355x.so
    CPL_LIB=$lib timeout -k 10 200 python -u scripts/solve_digest.py --batch $B > $O/digest_${t}_B$B.jsonl || exit $?
  done
done
bash scripts/ab_solve.sh $O/ab build/libcpl_pre_kkt.so centroidalplanner_amd/libcpl_mi355x.so
