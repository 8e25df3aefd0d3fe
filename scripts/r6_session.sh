#!/bin/bash
# Round 6 GPU session: the GPU suite, smoke(), the default bench line, then optional probes.
#   scripts/r6_session.sh OUT [sq8probe]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
if [ "$2" = sq8probe ]; then
  # sq8: full, no compute (1), no stores (2), no phase barriers (8192)
  timeout -k 10 300 python3 -u scripts/ab_kernels.py --config sq8 --rounds 5 --reps 20 \
    --variants 0:0:256:1,0:0:256:1:1,0:0:256:1:2,0:0:256:1:8192 > "$out/sq8_ablate.jsonl" || exit $?
  timeout -k 10 300 python3 -u scripts/ab_kernels.py --config sq16 --rounds 3 --reps 10 \
    --variants 0:0:256:1,0:0:256:1:1,0:0:256:1:2,0:0:256:1:8192 > "$out/sq16_ablate.jsonl" || exit $?
fi
echo done
