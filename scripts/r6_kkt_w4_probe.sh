#!/bin/bash
# Round 6: the one-wave KKT factorisation against its four-wave form (cpl_kkt_wave_kernel<47, 30, true>)
# — phase cycles, kernel time and the outputs' hash (bitwise) at B = 1 / 64 / 256 / 8 192.
# build/kprobe_base (the tree before) and build/kprobe_w4 (scripts/kkt_probe.hip on this tree; CPL_KKT_W4
# forces the form).   scripts/r6_kkt_w4_probe.sh OUT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=${1:?out dir}
mkdir -p "$out"
for B in 1 64 256 8192; do
  timeout -k 10 60 ./build/kprobe_base $B > "$out/base_$B.txt" || exit $?
  CPL_KKT_W4=1 timeout -k 10 60 ./build/kprobe_w4 $B > "$out/w4_$B.txt" || exit $?
  CPL_KKT_W4=0 timeout -k 10 60 ./build/kprobe_w4 $B > "$out/w1_$B.txt" || exit $?
done
echo done
