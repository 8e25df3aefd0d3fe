# round-5 GPU session: the kind split's Ground walker cap across the 1 / 2 / 4 / 8-GPU shard sizes
set -o pipefail
O=gpurun_out/r5_g9; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_entry_kernel.py tests/test_gpu_solve_engine.py -m gpu > $O/tests.log 2>&1 || exit $?
V=0:0:256:1:0,0:0:256:1:256,0:0:256:1:512
for B in 131072 262144 524288 1048576; do
  timeout -k 10 200 python -u scripts/ab_kernels.py --config mixed16 --batch $B --rounds 5 --reps 5 --variants $V --norms > $O/cap_$B.jsonl || exit $?
done
