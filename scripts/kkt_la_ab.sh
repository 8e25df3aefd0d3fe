#!/bin/bash
# A/B of the one-wave KKT kernel's QR look-ahead (scripts/kkt_probe) against the step-by-step QR
# (scripts/kkt_probe_nola, -DCPL_KKT_NO_LOOKAHEAD): kernel time, phase cycles and the outputs' hash
# at B = 1, 64 and 8192, interleaved.  usage: scripts/kkt_la_ab.sh OUTDIR
set -e
out=${1:-gpurun_out/kkt_la}
mkdir -p "$out"
for rep in 1 2; do
  for B in 1 64 8192; do
    timeout -k 5 60 ./scripts/kkt_probe_nola $B > "$out/nola_B${B}_r${rep}.txt"
    timeout -k 5 60 ./scripts/kkt_probe $B > "$out/la_B${B}_r${rep}.txt"
  done
done
grep -H "mode 0\|hash\|QR " "$out"/*.txt
