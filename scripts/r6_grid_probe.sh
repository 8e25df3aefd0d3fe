#!/bin/bash
# Round 6 (rejected, code reverted: the ablate 32768 bit it measured is gone): the pipelined / entry kernels' balanced persistent grid
# tiles) against min(tiles, resident) (ablate 32768), configs[1] and up.   scripts/r6_grid_probe.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
AB="python3 -u scripts/ab_kernels.py"
V="0:0:256:1,0:0:256:1:32768"
timeout -k 10 300 $AB --config ground4 --rounds 7 --reps 50 --variants $V --norms > "$out/ground4_65k.jsonl" || exit $?
timeout -k 10 300 $AB --config ground4 --batch 100003 --rounds 7 --reps 50 --variants $V --norms > "$out/ground4_100k.jsonl" || exit $?
timeout -k 10 300 $AB --config ground4 --batch 262144 --rounds 5 --reps 20 --variants $V --norms > "$out/ground4_262k.jsonl" || exit $?
timeout -k 10 300 $AB --config ground4_1m --rounds 5 --reps 10 --variants $V --norms > "$out/ground4_1m.jsonl" || exit $?
timeout -k 10 300 $AB --config none4 --rounds 5 --reps 20 --variants $V --norms > "$out/none4.jsonl" || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_north_star.py > "$out/tests.log" 2>&1 || exit $?
echo done
