"""The last dispatches of a rocprofv3 kernel trace as a timeline (start / end relative to the first
shown, microseconds): where a multi-kernel launch (the mixed kind split: partition, the two halves on
two streams, the norms' finish) spends its time.
usage: python scripts/trace_timeline.py <kernel_trace.csv> [count]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
cnt = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows = rows[-cnt:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    print(f"{s:10.1f} {e:10.1f} {e - s:9.1f}  q{r.get('Queue_Id', '?'):>3} grid {r['Grid_Size_X']:>9}  {name}")
