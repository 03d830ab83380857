"""Summarise a rocprofv3 kernel-trace (.db or *_kernel_stats.csv) into a small markdown/CSV
table under profiles/: kernel, calls, total us, average us, percent."""
import csv
import glob
import os
import sqlite3
import sys

src, out = sys.argv[1], sys.argv[2]
rows = []
# newest first: an output directory may hold earlier runs
dbs = sorted(glob.glob(os.path.join(src, "**", "*.db"), recursive=True), key=os.path.getmtime,
             reverse=True)
csvs = sorted(glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True),
              key=os.path.getmtime, reverse=True)
if csvs:
    for r in csv.DictReader(open(csvs[0])):
        rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                     float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
elif dbs:
    con = sqlite3.connect(dbs[0])
    for name, calls, tot, avg, pct in con.execute(
            "select name,total_calls,total_duration,average,percentage from top_kernels"):
        rows.append((name, calls, tot, avg, pct))  # top_kernels view is in us
with open(out, "w") as f:
    f.write("kernel,calls,total_us,avg_us,percent\n")
    for n, c, t, a, p in rows:
        f.write('"%s",%d,%.3f,%.3f,%.2f\n' % (n.split("(")[0], c, t, a, p))
print(open(out).read())
