# round-5 GPU session: the small-batch tail kernel (k_tail_small) — GPU suite, bitwise digests and
# solve A/B against the build before it
set -o pipefail
O=gpurun_out/r5_g28; mkdir -p $O/ab
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || exit $?
for B in 1 64 8192; do
  for t in A B; do
    lib=build/libcpl_pre_tail.so; [ $t = B ] && lib=centroidalplanner_amd/libcpl_mi355x.so
    CPL_LIB=$lib timeout -k 10 200 python -u scripts/solve_digest.py --batch $B > $O/digest_${t}_B$B.jsonl || exit $?
  done
done
bash scripts/ab_solve.sh $O/ab build/libcpl_pre_tail.so centroidalplanner_amd/libcpl_mi355x.so
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o run -- \
  python3 scripts/solve_latency.py --reps 5 --only limited-memory:1 > $O/prof_b1.log 2>&1
