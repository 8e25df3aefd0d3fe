#!/bin/bash
# the kind split: the partition's scan folded into the write kernel (mixed-batch parity tests), and
# the Ground list budget (40 default; 48 / 36 / 32 KiB) on the 50/50 mixed batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:-gpurun_out/g25}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_entry_kernel.py tests/test_gpu_parity.py -m gpu > "$out/tests.log" 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_kernels.py --config mixed16 --rounds 4 --reps 5 --variants 0:0:256:1,0:0:256:1:16,0:0:256:1:64,0:0:256:1:128,0:0:256:1:96 --norms > "$out/mixed16_list_lds.jsonl"
