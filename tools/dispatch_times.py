"""Per-dispatch durations (us) of the mmt kernels in a rocprofv3 results db, grouped by kernel
and grid shape: python tools/dispatch_times.py gpurun_out/orbk/run_results.db"""
import sqlite3
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
acc = defaultdict(list)
for name, gx, gy, gz, dur in con.execute(
        "select name, grid_x, grid_y, grid_z, duration from kernels where name like '%mmt::%'"):
    acc[(name.split("(")[0], gx, gy, gz)].append(dur / 1e3)
for (n, gx, gy, gz), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print("%-22s grid %6d x %4d x %3d  n=%3d  median %8.2f us  min %8.2f" %
          (n, gx, gy, gz, len(v), v[len(v) // 2], v[0]))
