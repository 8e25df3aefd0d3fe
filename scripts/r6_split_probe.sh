#!/bin/bash
# Round 6: where the mixed kind split's time goes (GPU box).  Same-process timings of the split, its
# halves alone and the non-list kernels of the same records; a kernel trace of the split (timeline of
# the two halves); SQ wait / instruction counters per kernel (each pass its own rocprofv3 run).
#   scripts/r6_split_probe.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
AB="python3 -u scripts/ab_kernels.py"
(cd /tmp && timeout -k 10 60 rocprofv3 -L) > "$out/counters_avail.txt" 2>&1
# 0 = default split, 4 = halves one after the other on one stream, 256 = Ground walkers uncapped
timeout -k 10 300 $AB --config mixed16 --rounds 3 --reps 10 --variants 0:0:256:1,0:0:256:1:4,0:0:256:1:256 > "$out/mixed16.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 10 --variants 0:0:256:1 > "$out/list_sq_524k.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 524288 --tags all_ground --rounds 3 --reps 10 --variants 0:0:256:1 > "$out/list_ground_524k.jsonl" || exit $?
timeout -k 10 200 $AB --config sq16 --rounds 3 --reps 10 --variants 0:0:256:1 > "$out/sq16.jsonl" || exit $?
timeout -k 10 200 $AB --config ground16 --rounds 3 --reps 10 --variants 0:0:256:1 > "$out/ground16.jsonl" || exit $?
cd /tmp || exit 1
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/kt" -o k -- \
  python3 "$R/scripts/ab_kernels.py" --config mixed16 --rounds 1 --reps 3 --variants 0:0:256:1 > "$R/$out/kt.log" 2>&1 || exit $?
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
P2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  for cfg in mixed16 sq16 sq8; do
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$R/$out/pmc_$cfg/p$i" -o p -- \
      python3 "$R/scripts/ab_kernels.py" --config $cfg --rounds 1 --reps 2 --variants 0:0:256:1 > "$R/$out/pmc_${cfg}_p$i.log" 2>&1 || exit $?
  done
done
echo done
