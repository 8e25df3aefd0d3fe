# round-5 GPU session: the committed priority changes against the tree before them + Superquadric / mixed GPU tests
set -o pipefail
O=gpurun_out/r5_g40; mkdir -p $O
bash scripts/ab_eval.sh $O build/libcpl_pre_prio.so centroidalplanner_amd/libcpl_mi355x.so sq8 sq16 mixed16 "mixed16:--batch 131072" || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu -k "sq or superquadric or parity or mixed or split" > $O/tests.log 2>&1
