# round-5 GPU session: the committed side-stream priority — split / mixed GPU tests and the A/B
set -o pipefail
O=gpurun_out/r5_g47; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu -k "mixed or split or entry or graph" > $O/tests.log 2>&1 || exit $?
bash scripts/ab_eval.sh $O build/libcpl_pre_prio.so centroidalplanner_amd/libcpl_mi355x.so mixed16 "mixed16:--batch 131072" || exit $?
