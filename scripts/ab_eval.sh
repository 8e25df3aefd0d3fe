#!/bin/bash
# Same-process A/B of two builds of the HIP library on eval configs (scripts/ab_libs.py: interleaved
# rounds, HIP-event kernel time, outputs compared bit for bit).  Run on the GPU box:
#   scripts/ab_eval.sh <out dir> <lib A> <lib B> <config[:extra ab_libs args]> ...
# e.g. scripts/ab_eval.sh gpurun_out/ab_sq centroidalplanner_amd/libcpl_mi355x.so build/libcpl_r4.so sq8 mixed16
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=$1; a=$2; b=$3; shift 3
mkdir -p "$out"
for spec in "$@"; do
  cfg=${spec%%:*}; extra=""
  [ "$spec" != "$cfg" ] && extra=${spec#*:}
  tag=$(echo "$spec" | tr ' :' '__')
  timeout -k 10 300 python -u scripts/ab_libs.py --config "$cfg" --rounds 5 --reps 10 --libs "$a,$b" $extra \
    > "$out/$tag.jsonl" 2> "$out/$tag.err" || exit $?
done
