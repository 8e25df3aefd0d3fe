"""Per (kernel, grid size) call counts and mean durations from a rocprofv3 kernel trace.

The bench runs several launch shapes in one process (the timed 1M-instance launches, the 65k
side field, the single-instance latency probe, the checker): rocprof's --stats averages them
together.  This splits the trace by grid so the timed kernel's average can be compared with the
bench's HIP-event kernel_ms.
usage: python scripts/trace_by_grid.py <run_kernel_trace.csv> [out.csv]
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0], int(r["Grid_Size_X"]),
           int(r["Workgroup_Size_X"]))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = [("kernel", "grid_x", "workgroup_x", "calls", "mean_us", "min_us", "max_us", "total_ms")]
for (k, g, w), d in sorted(agg.items(), key=lambda t: -sum(t[1])):
    out.append((k, g, w, len(d), round(sum(d) / len(d), 3), round(min(d), 3), round(max(d), 3), round(sum(d) / 1e3, 3)))
if len(sys.argv) > 2:
    csv.writer(open(sys.argv[2], "w", newline="")).writerows(out)
for r in out[:15]:
    print(*r, sep="\t")
