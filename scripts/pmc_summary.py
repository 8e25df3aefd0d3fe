"""Summarise rocprofv3 --pmc CSV passes (scripts/pmc_eval.sh output dirs) per kernel: the mean counter
value per dispatch of every kernel whose name matches a pattern.
    python scripts/pmc_summary.py <dir with a/ b/ c/ ...> [kernel substring]"""
import csv
import glob
import os
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "tile_kernel"
agg = {}
for f in sorted(glob.glob(os.path.join(root, "*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
