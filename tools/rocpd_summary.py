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
ap.add_argument("--mmt-only", action="store_true", help="only the mmt:: kernels (and the runtime's copies)")
ap.add_argument("--orb-window", type=int, default=0,
                help="also report the span of every batched ORB window of this batch size: from "
                     "its k_gray_depth start to the last ORB kernel's end")
a = ap.parse_args()
db = a.src
if os.path.isdir(db):
    db = sorted(glob.glob(os.path.join(db, "**", "*.db"), recursive=True), key=os.path.getmtime)[-1]
con = sqlite3.connect(db)
where = " where name like '%mmt::%' or name like '%rocclr%'" if a.mmt_only else ""
rows = con.execute("select name, duration, grid_x, grid_y, grid_z from kernels%s order by start"
                   % where).fetchall()
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

if a.orb_window:
    orb = ("k_gray_depth", "k_resize", "k_pyramid", "k_fast", "k_octree", "k_blur", "k_orient_desc")
    rows = [r for r in con.execute("select name, start, end, grid_y from kernels where name like "
                                   "'%k_gray_depth%' or name like '%k_resize%' or name like "
                                   "'%k_pyramid%' or name like '%k_fast%' or name like '%k_octree%'"
                                   " or name like '%k_blur%' or name like '%k_orient_desc%' "
                                   "order by start")]
    spans, t0, end = [], None, 0
    for nm, st, en, gy in rows:  # one pass: a window opens at each batched k_gray_depth
        if "k_gray_depth" in nm and gy == a.orb_window:
            if t0 is not None:
                spans.append((end - t0) / 1e3)
            t0, end = st, en
        elif t0 is not None:
            end = max(end, en)
    if t0 is not None:
        spans.append((end - t0) / 1e3)
    if spans:
        sp = sorted(spans)
        print("ORB windows at batch %d: %d, mean %.1f us, median %.1f us, min %.1f us"
              % (a.orb_window, len(sp), sum(sp) / len(sp), sp[len(sp) // 2], sp[0]))
