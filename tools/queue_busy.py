"""Per-queue busy time of the mmt:: kernels in a rocprofv3 kernel trace over its last `window_ms`,
and per (queue, kernel) count and mean duration: which chain of the tracker is the critical one.
Usage: queue_busy.py <trace dir> [window_ms]"""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
window_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
f = sorted(glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True),
           key=os.path.getmtime)[-1]
ks = []
for r in csv.DictReader(open(f)):
    name = r.get("Kernel_Name", r.get("KernelName", ""))
    if "mmt::" not in name:
        continue
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q,
               name.split("(")[0].replace("void ", "").replace("mmt::", "")))
ks.sort()
end = ks[-1][1]
t0 = end - window_ms * 1e6
busy = collections.Counter()
per = collections.defaultdict(list)
for s, e, q, n in ks:
    if s < t0:
        continue
    busy[q] += e - s
    per[(q, n)].append(e - s)
print("window %.1f ms" % window_ms)
for q, b in sorted(busy.items()):
    print("queue %s busy %.1f%%" % (q, 100 * b / (window_ms * 1e6)))
    for (qq, n), v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        if qq == q and sum(v) > 0.01 * b:
            print("   %-28s n=%5d mean %8.1f us  total %6.1f%%" % (
                n, len(v), sum(v) / len(v) / 1e3, 100 * sum(v) / b))
