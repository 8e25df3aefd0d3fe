# round-5 GPU session: the Ground backtracking kernel held to 128 VGPRs (four waves per SIMD) — digests and
# the solve A/B
set -o pipefail
O=gpurun_out/r5_g45; mkdir -p $O/ab
for B in 1 64 8192; do
  for t in A B; do
    lib=centroidalplanner_amd/libcpl_mi355x.so; [ $t = B ] && lib=build/libcpl_ls4.so
    CPL_LIB=$lib timeout -k 10 200 python -u scripts/solve_digest.py --batch $B > $O/digest_${t}_B$B.jsonl || exit $?
  done
done
bash scripts/ab_solve.sh $O/ab centroidalplanner_amd/libcpl_mi355x.so build/libcpl_ls4.so
