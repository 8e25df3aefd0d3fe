"""Per-kernel summary of a rocprofv3 SQLite trace (rocpd *_results.db): name, grid, calls, mean/min
duration.  python scripts/rocpd_summary.py <db> [--csv out.csv]"""
import csv
import sqlite3
import sys


def summary(db):
    con = sqlite3.connect(db)
    cur = con.cursor()
    rows = cur.execute(
        "select s.display_name, d.grid_size_x, d.workgroup_size_x, d.end - d.start "
        "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    agg = {}
    order = []
    for name, grid, wg, dur in rows:
        key = (name, grid, wg)
        if key not in agg:
            agg[key] = []
            order.append(key)
        agg[key].append(dur)
    out = []
    for key in order:
        ds = agg[key]
        out.append({"kernel": key[0][:90], "grid": key[1], "wg": key[2], "calls": len(ds),
                    "mean_us": sum(ds) / len(ds) / 1e3, "min_us": min(ds) / 1e3})
    return out


if __name__ == "__main__":
    res = summary(sys.argv[1])
    for r in res:
        print(f"{r['calls']:5d} {r['mean_us']:10.1f} us (min {r['min_us']:9.1f})  grid {r['grid']:9d} wg {r['wg']:4d}  {r['kernel']}")
    if "--csv" in sys.argv:
        with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(res[0].keys()))
            w.writeheader()
            w.writerows(res)
