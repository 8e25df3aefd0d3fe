# round-5 GPU session: the KKT wave kernel's changes without the twelve-per-CU form (CPL_KKT_NO_ZG) against
# the build before them
set -o pipefail
O=gpurun_out/r5_g31; mkdir -p $O/ab
export CPL_KKT_NO_ZG=1
for B in 8192; do
  for t in A B; do
    lib=build/libcpl_pre_kkt.so; [ $t = B ] && lib=centroidalplanner_amd/libcpl_mi355x.so
    CPL_LIB=$lib timeout -k 10 200 python -u scripts/solve_digest.py --batch $B > $O/digest_${t}_B$B.jsonl || exit $?
  done
done
bash scripts/ab_solve.sh $O/ab build/libcpl_pre_kkt.so centroidalplanner_amd/libcpl_mi355x.so
