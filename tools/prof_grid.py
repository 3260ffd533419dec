"""Per-launch durations of a rocprofv3 kernel trace (rocpd SQLite database) binned by
grid size: how each kernel's time grows with the batch.  usage: prof_grid.py DIR [substr...]"""
import glob
import os
import sqlite3
import sys

db = glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True)[0]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
gcol = next((k for k in ("grid_size", "grid_x", "grid_size_x", "workgroup_count") if k in cols), None)
print("columns:", ",".join(cols))
if gcol is None:
    sys.exit(0)
pats = sys.argv[2:] or [""]
rows = c.execute(f"select name, {gcol}, duration from kernels").fetchall()
for p in pats:
    sel = [(n, g, d) for n, g, d in rows if p in n]
    names = sorted({n for n, _, _ in sel})
    for n in names:
        by = {}
        for nn, g, d in sel:
            if nn == n:
                b = 1 << max(0, int(g).bit_length() - 1)
                by.setdefault(b, []).append(d)
        print(n[:90])
        for b in sorted(by):
            v = by[b]
            print(f"   grid >= {b:8d}: {len(v):5d} launches, avg {sum(v) / len(v) / 1e3:8.1f} us, max {max(v) / 1e3:8.1f} us")
