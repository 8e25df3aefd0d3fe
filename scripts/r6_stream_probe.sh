#!/bin/bash
# Round 6: mixed16's box-to-box spread (2.21-2.42 ms) against the streams' hardware queues —
# scripts/mixed_stream_probe.py at 1 048 576 and 131 072 x 16, then the bench line twice.
# scripts/r6_stream_probe.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
timeout -k 10 300 python3 -u scripts/mixed_stream_probe.py > "$out/streams_1m.jsonl" || exit $?
timeout -k 10 200 python3 -u scripts/mixed_stream_probe.py --batch 131072 --reps 40 > "$out/streams_131k.jsonl" || exit $?
timeout -k 10 300 python3 -u bench.py --config mixed16 > "$out/bench_mixed16_a.json" 2> "$out/bench_a.err" || exit $?
timeout -k 10 300 python3 -u bench.py --config mixed16 --no-pmc > "$out/bench_mixed16_b.json" 2> "$out/bench_b.err" || exit $?
echo done
