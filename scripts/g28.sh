#!/bin/bash
# the kind split's new defaults (Ground grid one per CU, Superquadric tiles at 40 KiB) against the
# previous ones (ablation 256 | 32), on the 50/50, all-Ground and all-Superquadric mixed batches; the
# mixed-batch parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g28}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_entry_kernel.py tests/test_gpu_parity.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
V=0:0:256:1,0:0:256:1:32,0:0:256:1:256,0:0:256:1:512
timeout -k 10 300 python -u scripts/ab_kernels.py --config mixed16 --rounds 4 --reps 5 --variants $V --norms > "$out/mixed16.jsonl" || exit $?
timeout -k 10 300 python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_ground --rounds 3 --reps 5 --variants $V --norms > "$out/allground.jsonl" || exit $?
timeout -k 10 300 python -u scripts/ab_kernels.py --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 5 --variants $V --norms > "$out/allsq.jsonl"
