set -o pipefail
O=gpurun_out/r5_g2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sq_sweep.py tests/test_gpu_entry_kernel.py tests/test_golden.py -m gpu > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/ab_kernels.py --config sq8 --rounds 5 --reps 10 --variants 0:0:256:1:0,0:0:256:1:1024 --norms > $O/sq8.jsonl || exit $?
timeout -k 10 200 python -u scripts/ab_kernels.py --config sq16 --rounds 5 --reps 10 --variants 0:0:256:1:0,0:0:256:1:1024 --norms > $O/sq16.jsonl || exit $?
timeout -k 10 300 python -u scripts/ab_kernels.py --config mixed16 --rounds 4 --reps 5 --variants 0:0:256:1:0,0:0:256:1:1024,0:0:256:1:2048 --norms > $O/mixed16.jsonl || exit $?
scripts/pmc_eval.sh sq8 $O/pmc_sq8_nopt 0:0:256:1:1024
