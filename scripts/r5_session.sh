# round-5 GPU session: the mixed split with / without the uniform-axis mapping in its Superquadric half
set -o pipefail
O=gpurun_out/r5_g5; mkdir -p $O
L=centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_nouax_list.so,build/libcpl_r4.so
timeout -k 10 300 python -u scripts/ab_libs.py --config mixed16 --rounds 7 --reps 5 --libs $L > $O/mixed16.jsonl || exit $?
timeout -k 10 200 python -u scripts/ab_libs.py --config mixed16 --batch 131072 --rounds 7 --reps 10 --libs $L > $O/mixed16_131k.jsonl
