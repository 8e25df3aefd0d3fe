# round-5 GPU session: the SQST build's GPU tests, then the phase ablations on it (measurement-only build)
set -o pipefail
O=gpurun_out/r5_g19; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || exit $?
V=0:0:256:1:0,0:0:256:1:2048,0:0:256:1:4096,0:0:256:1:8192,0:0:256:1:16384,0:0:256:1:30720,0:0:256:1:1,0:0:256:1:2
for c in sq8 sq16; do
CPL_LIB=build/libcpl_abl2.so timeout -k 10 300 python -u scripts/ab_kernels.py --config $c --rounds 5 --reps 10 --variants $V --norms > $O/${c}_phases.jsonl || exit $?
done
