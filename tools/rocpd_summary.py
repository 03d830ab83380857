"""Per-kernel summary of a rocprofv3 results database (rocpd SQLite, the default output of
`rocprofv3 --kernel-trace`): calls, total and average duration per kernel name, optionally split
by grid size.  Usage: rocpd_summary.py <dir-or-db> [--by-grid] [--skip N] (skip the first N
dispatches of every kernel: warm-up)."""
import argparse
import collections
import glob
import os
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("--by-grid", action="store_true")
ap.add_argument("--skip", type=int, default=0)
a = ap.parse_args()
db = a.src
if os.path.isdir(db):
    db = sorted(glob.glob(os.path.join(db, "**", "*.db"), recursive=True), key=os.path.getmtime)[-1]
con = sqlite3.connect(db)
rows = con.execute("select name, duration, grid_x, grid_y, grid_z from kernels order by start").fetchall()
acc = collections.OrderedDict()
seen = collections.Counter()
for name, dur, gx, gy, gz in rows:
    short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "")
    seen[short] += 1
    if seen[short] <= a.skip:
        continue
    key = (short, (gx, gy, gz)) if a.by_grid else (short, None)
    n, t = acc.get(key, (0, 0))
    acc[key] = (n + 1, t + dur)
tot = sum(t for n, t in acc.values())
print("%-34s %-20s %6s %12s %10s %6s" % ("kernel", "grid", "calls", "total_us", "avg_us", "pct"))
for (k, g), (n, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
    print("%-34s %-20s %6d %12.1f %10.2f %6.2f" % (k[:34], "" if g is None else "x".join(map(str, g)),
                                                  n, t / 1e3, t / 1e3 / n, 100.0 * t / tot))
