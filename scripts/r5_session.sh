# round-5 GPU session: the split's Ground walker cap with the high-priority side stream (ablate 256 = every
# Ground workgroup walking, 512 = two per CU; default one per CU)
set -o pipefail
O=gpurun_out/r5_g48; mkdir -p $O
A=centroidalplanner_amd/libcpl_mi355x.so; B=build/libcpl_same.so
for tun in 0:0:256:1:0 0:0:256:1:256 0:0:256:1:512; do
  for spec in "mixed16" "mixed16 --batch 262144"; do
    tag=$(echo "$tun $spec" | tr ' :' '__')
    timeout -k 10 300 python -u scripts/ab_libs.py --config $spec --rounds 5 --reps 10 --libs "$A,$B" --tuning $tun \
      > $O/$tag.jsonl 2> $O/$tag.err || exit $?
  done
done
