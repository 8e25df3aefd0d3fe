# round-5 GPU session: Superquadric batches through the pipelined kernel on four compute waves + the
# loader (variant 2 = VAR_PIPE) against the tile kernel (variant 0); in-tree = generic row items,
# build/libcpl_sqpipe_af.so = axis-specialised row items
set -o pipefail
O=gpurun_out/r5_g33; mkdir -p $O
A=centroidalplanner_amd/libcpl_mi355x.so; B=build/libcpl_sqpipe_af.so
for tun in 0:0:256:1 2:0:256:1; do
  for cfg in sq8 sq16; do
    timeout -k 10 300 python -u scripts/ab_libs.py --config $cfg --rounds 5 --reps 10 --libs "$A,$B" --tuning $tun \
      > $O/${cfg}_$tun.jsonl 2> $O/${cfg}_$tun.err || exit $?
  done
done
