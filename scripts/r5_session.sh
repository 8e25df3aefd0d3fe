# round-5 GPU session: the loader wave of the pipelined and entry kernels at raised priority
set -o pipefail
O=gpurun_out/r5_g41; mkdir -p $O
bash scripts/ab_eval.sh $O centroidalplanner_amd/libcpl_mi355x.so build/libcpl_ldr.so ground4_1m ground4 ground16 mixed16 none4 || exit $?
