"""Summarize a rocprofv3 kernel trace (rocpd SQLite database or kernel_stats.csv) as
the per-kernel stats table committed under profiles/ (Name, Calls, Total, Average)."""
import csv
import glob
import os
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
         "from kernels group by name order by sum(duration) desc")
    return [list(r) for r in c.execute(q)]


def main(src, out):
    if os.path.isdir(src):
        dbs = glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
        src = dbs[0]
    rows = rows_from_db(src)
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, s, a, mn, mx in rows:
            w.writerow([name, n, s, round(a, 1), round(100.0 * s / total, 2), mn, mx])
    for name, n, s, a, *_ in rows:
        print(f"{name[:90]:90s} {n:6d} {a / 1e3:10.1f} us {s / 1e6:9.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
