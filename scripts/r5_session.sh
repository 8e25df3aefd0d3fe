# round-5 GPU session: the new small-batch-tail equivalence test
set -o pipefail
O=gpurun_out/r5_g34; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_solve_engine.py -m gpu > $O/t.log 2>&1
