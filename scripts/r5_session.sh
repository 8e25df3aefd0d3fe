# round-5 GPU session: the priority changes against the tree before them with the library order swapped
# (ab_libs' second library measured ~3 % faster on sq8 even when both are the same build)
set -o pipefail
O=gpurun_out/r5_g44; mkdir -p $O/ab $O/ba $O/same
bash scripts/ab_eval.sh $O/ab build/libcpl_pre_prio.so centroidalplanner_amd/libcpl_mi355x.so sq8 sq16 mixed16 "mixed16:--tags all_sq" || exit $?
bash scripts/ab_eval.sh $O/ba centroidalplanner_amd/libcpl_mi355x.so build/libcpl_pre_prio.so sq8 sq16 mixed16 "mixed16:--tags all_sq" || exit $?
cp centroidalplanner_amd/libcpl_mi355x.so /tmp/libcpl_copy.so
bash scripts/ab_eval.sh $O/same centroidalplanner_amd/libcpl_mi355x.so /tmp/libcpl_copy.so sq8 || exit $?
