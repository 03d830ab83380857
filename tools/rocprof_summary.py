"""Summarise a rocprofv3 kernel-trace (.db or *_kernel_stats.csv) into a small CSV table under
profiles/: kernel, calls, total us, average us, percent.  A third argument `mmt` keeps only the
library's kernels (mmt::, the bench's synthetic-scene rendering and torch copies dropped) with the
percent recomputed over them; an existing summary CSV is accepted as the source too.
Usage: rocprof_summary.py <rocprof dir | summary.csv> <out.csv> [mmt]"""
import csv
import glob
import os
import sqlite3
import sys

src, out = sys.argv[1], sys.argv[2]
only_mmt = len(sys.argv) > 3 and sys.argv[3] == "mmt"
rows = []
# newest first: an output directory may hold earlier runs
dbs = sorted(glob.glob(os.path.join(src, "**", "*.db"), recursive=True), key=os.path.getmtime,
             reverse=True)
csvs = sorted(glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True),
              key=os.path.getmtime, reverse=True)
if src.endswith(".csv") and os.path.isfile(src):  # an earlier summary of this tool
    for r in csv.DictReader(open(src)):
        rows.append((r["kernel"], int(r["calls"]), float(r["total_us"]), float(r["avg_us"]),
                     float(r["percent"])))
elif csvs:
    for r in csv.DictReader(open(csvs[0])):
        rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                     float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
elif dbs:
    con = sqlite3.connect(dbs[0])
    for name, calls, tot, avg, pct in con.execute(
            "select name,total_calls,total_duration,average,percentage from top_kernels"):
        rows.append((name, calls, tot, avg, pct))  # top_kernels view is in us
if only_mmt:
    rows = [r for r in rows if "mmt::" in r[0]]
    tot = sum(r[2] for r in rows) or 1.0
    rows = sorted(((n, c, t, a, 100.0 * t / tot) for n, c, t, a, _ in rows), key=lambda r: -r[2])
with open(out, "w") as f:
    f.write("kernel,calls,total_us,avg_us,percent\n")
    for n, c, t, a, p in rows:
        f.write('"%s",%d,%.3f,%.3f,%.2f\n' % (n.replace("(anonymous namespace)::", "").split("(")[0],
                                                c, t, a, p))
print(open(out).read())
