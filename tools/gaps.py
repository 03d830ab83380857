"""Idle analysis of a rocprofv3 kernel trace: over the last `window_ms`, list the intervals where
no mmt:: kernel runs on any queue (longer than `min_us`), and the union busy fraction."""
import csv
import glob
import os
import sys

src = sys.argv[1]
window_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 40.0
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
f = sorted(glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True),
           key=os.path.getmtime)[-1]
ks = []
for r in csv.DictReader(open(f)):
    name = r.get("Kernel_Name", r.get("KernelName", ""))
    if "mmt::" not in name:
        continue
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0]))
ks.sort()
end = ks[-1][1]
t0 = end - window_ms * 1e6
ks = [k for k in ks if k[0] >= t0]
busy_until = ks[0][0]
busy = 0
gaps = []
for s, e, n in ks:
    if s > busy_until:
        gaps.append((busy_until, s, n))
    if e > busy_until:
        busy += e - max(s, busy_until)
        busy_until = e
span = ks[-1][1] - ks[0][0]
print("window %.1f ms, union busy %.1f %%, kernels %d" % (span / 1e6, 100.0 * busy / span, len(ks)))
for a, b, n in gaps:
    if (b - a) / 1e3 >= min_us:
        print("idle %8.1f us at %9.1f us before %s" % ((b - a) / 1e3, (a - ks[0][0]) / 1e3, n))
