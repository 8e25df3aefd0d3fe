# round-5 GPU session: the GPU suite with the engine's NLP scaling, TestBasic's outcomes, solve benches
set -o pipefail
O=gpurun_out/r5_g10; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/testbasic_outcomes.py gpu > $O/testbasic_gpu.jsonl 2> $O/testbasic_gpu.err || exit $?
timeout -k 10 300 python -u bench.py --config solve5 --hessian limited-memory > $O/bench_solve5_lm.json 2> $O/bench_solve5_lm.err || exit $?
timeout -k 10 300 python -u bench.py --config solve5 > $O/bench_solve5.json 2> $O/bench_solve5.err || exit $?
timeout -k 10 200 python -u scripts/solve_latency.py > $O/solve_latency.txt 2>&1 || exit $?
