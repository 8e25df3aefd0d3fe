# round-5 GPU session: uniform-axis row items in the kind split's Superquadric list tiles (with / without a 4-wave cap)
set -o pipefail
O=gpurun_out/r5_g14; mkdir -p $O
L=centroidalplanner_amd/libcpl_mi355x.so,build/libcpl_lu.so,build/libcpl_lu_cap.so
timeout -k 10 300 python -u scripts/ab_libs.py --config mixed16 --rounds 5 --reps 10 --libs $L > $O/mixed16.jsonl 2> $O/mixed16.err || exit $?
timeout -k 10 300 python -u scripts/ab_libs.py --config mixed16 --rounds 5 --reps 10 --libs $L --tags all_sq > $O/mixed16_allsq.jsonl 2> $O/allsq.err || exit $?
timeout -k 10 300 python -u scripts/ab_libs.py --config sq8 --rounds 5 --reps 10 --libs $L > $O/sq8.jsonl 2> $O/sq8.err || exit $?
