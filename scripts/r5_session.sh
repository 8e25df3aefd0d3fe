# round-5 GPU session: the GPU suite after the engine-side NaN count, then the plain-double power-ladder A/B
set -o pipefail
O=gpurun_out/r5_g11; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit $?
bash scripts/ab_eval.sh $O/plain centroidalplanner_amd/libcpl_mi355x.so build/libcpl_plain.so sq8 sq16 mixed16
