# round-5 GPU session: raised wave priority around the copy phases of Superquadric tiles of 8+ instances
set -o pipefail
O=gpurun_out/r5_g38; mkdir -p $O
bash scripts/ab_eval.sh $O build/libcpl_pre_prio.so centroidalplanner_amd/libcpl_mi355x.so sq8 sq16 mixed16 "sq8:--batch 20000" || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu -k "sq or superquadric or parity or mixed" > $O/tests.log 2>&1
