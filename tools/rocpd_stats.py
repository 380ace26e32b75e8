#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 --kernel-trace run, split by launch grid (so a kernel
launched at two batch sizes gets two rows): Name, grid, calls, total / average / min / max
duration in ns. Input: the SQLite database (rocpd, the default output) or the
`*_kernel_trace.csv` of --output-format csv.
usage: python tools/rocpd_stats.py <results.db | kernel_trace.csv> <out.csv>"""
import csv
import sqlite3
import sys


def from_trace_csv(path):
    agg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            key = (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            agg.setdefault(key, []).append(d)
    rows = [(n, gx, gy, len(v), sum(v) / len(v), sum(v), min(v), max(v))
            for (n, gx, gy), v in agg.items()]
    return sorted(rows, key=lambda r: -r[5])


def main():
    db, out = sys.argv[1], sys.argv[2]
    if db.endswith(".csv"):
        rows = from_trace_csv(db)
    else:
        c = sqlite3.connect(db)
        rows = c.execute("select name, grid_x, grid_y, count(*), avg(end-start), sum(end-start), "
                         "min(end-start), max(end-start) from kernels group by name, grid_x, "
                         "grid_y order by sum(end-start) desc").fetchall()
    tot = sum(r[5] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "GridX", "GridY", "Calls", "TotalDurationNs", "AverageNs",
                    "Percentage", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], r[3], r[5], round(r[4], 1), round(100 * r[5] / tot, 2),
                        r[6], r[7]])


if __name__ == "__main__":
    main()
