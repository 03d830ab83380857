"""Critical-chain analysis of a rocprofv3 kernel trace of bench.py: on the queue whose
k_flow_lm launches are the longest (D3, PoseOptimizationFlow2 of the objects), the mean D3
duration, the mean idle-plus-other time between consecutive D3 launches, and what runs on that
queue in between.  Usage: d3_gaps.py <trace dir>"""
import collections
import csv
import glob
import os
import sys

import numpy as np

f = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True),
           key=os.path.getmtime)[-1]
ks = []
for r in csv.DictReader(open(f)):
    n = r.get("Kernel_Name", "")
    if "mmt::" not in n:
        continue
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"),
               n.split("(")[0].replace("void ", "").replace("mmt::", "")))
ks.sort()
q = collections.defaultdict(list)
for s, e, qq, n in ks:
    if n.startswith("k_flow_lm"):
        q[qq].append(e - s)
d3q = max(q, key=lambda k: sum(q[k]) / len(q[k]))
seq = [(s, e, n) for s, e, qq, n in ks if qq == d3q][-600:]
gaps, lm, between = [], [], collections.defaultdict(list)
last_end, acc = None, collections.Counter()
for s, e, n in seq:
    if n.startswith("k_flow_lm"):
        if last_end is not None:
            gaps.append(s - last_end)
            for k, v in acc.items():
                between[k].append(v)
        acc = collections.Counter()
        lm.append(e - s)
        last_end = e
    elif last_end is not None:
        acc[n] += e - s
print("D3 queue %s: k_flow_lm mean %.1f us; end-to-start gap to the next D3 mean %.1f us "
      "(median %.1f)" % (d3q, np.mean(lm) / 1e3, np.mean(gaps) / 1e3, np.median(gaps) / 1e3))
for k, v in sorted(between.items(), key=lambda kv: -np.mean(kv[1])):
    print("   %-22s %6.1f us per gap" % (k, np.mean(v) / 1e3))
g = np.array(gaps) / 1e3
print("gap percentiles (us): p50 %.0f p75 %.0f p90 %.0f p95 %.0f p99 %.0f max %.0f; gaps > 300 us: "
      "%d of %d, their share of the total gap time %.0f%%" % (
          np.percentile(g, 50), np.percentile(g, 75), np.percentile(g, 90), np.percentile(g, 95),
          np.percentile(g, 99), g.max(), (g > 300).sum(), len(g), 100 * g[g > 300].sum() / g.sum()))
big = [i for i, v in enumerate(g) if v > 300]
print("indices of gaps > 300 us:", big[:40])
