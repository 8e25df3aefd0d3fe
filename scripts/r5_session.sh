# round-5 GPU session: every list row in 16-byte DMA granules (shifted slots) — A/B against the in-tree build
set -o pipefail
O=gpurun_out/r5_g25; mkdir -p $O
bash scripts/ab_eval.sh $O/shift centroidalplanner_amd/libcpl_mi355x.so build/libcpl_shift.so mixed16 "mixed16:--tags all_ground" "mixed16:--batch 131072" || exit $?
