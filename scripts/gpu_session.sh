#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box; each step has its own time limit and the
# session stops at the first fault / abort / time-out (exit >= 124), never retrying.
# usage: scripts/gpu_session.sh "<secs> <cmd...>" "<secs> <cmd...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
log=gpurun_out/steps.log
: > "$log"
for step in "$@"; do
  secs=${step%% *}
  cmd=${step#* }
  echo "=== [$(date +%T)] $cmd" | tee -a "$log"
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "=== rc=$rc" | tee -a "$log"
  if [ "$rc" -ge 124 ]; then
    echo "stopping: fault/abort/timeout" | tee -a "$log"
    exit "$rc"
  fi
done
exit 0
