#!/bin/bash
# Round 6: the LDS-staged uniform-axis list tiles (variant 6) — their priority knob (ablate 4096), the
# division-free row copy-out; kernel trace and SQ counters of the variant-6 split.   scripts/r6_split_probe3.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
AB="python3 -u scripts/ab_kernels.py"
V="0:0:256:1,6:0:256:1,6:0:256:1:4096"
timeout -k 10 200 python3 -u scripts/variant_bitwise.py --config mixed16 --batch 20011 --variants 6:0:256:1,6:0:256:1:4096 > "$out/bitwise.jsonl" || exit $?
timeout -k 10 400 $AB --config mixed16 --rounds 4 --reps 10 --variants $V > "$out/mixed16.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 131072 --rounds 4 --reps 20 --variants $V > "$out/mixed16_shard.jsonl" || exit $?
timeout -k 10 200 $AB --config mixed16 --batch 524288 --tags all_sq --rounds 3 --reps 10 --variants $V > "$out/list_sq_524k.jsonl" || exit $?
timeout -k 10 200 $AB --config sq16 --rounds 3 --reps 10 --variants 0:0:256:1 > "$out/sq16.jsonl" || exit $?
cd /tmp || exit 1
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/kt" -o k -- \
  python3 "$R/scripts/ab_kernels.py" --config mixed16 --rounds 1 --reps 3 --variants 6:0:256:1 > "$R/$out/kt.log" 2>&1 || exit $?
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
P2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$R/$out/pmc_v6/p$i" -o p -- \
    python3 "$R/scripts/ab_kernels.py" --config mixed16 --rounds 1 --reps 2 --variants 6:0:256:1 > "$R/$out/pmc_v6_p$i.log" 2>&1 || exit $?
done
echo done
