"""Steady-state view of the tracker's three device chains from a rocprofv3 kernel trace: for each
queue, the period between consecutive launches of its marker kernel (ego: k_flow_lm_split or
k_pose_opt_l; D3: k_flow_lm; RANSAC: k_pnp_hyp), the mean duration of every kernel per frame, and
the busy fraction, over the middle of the run (first and last 10 % of the markers dropped).
Usage: chains.py <trace dir>"""
import collections
import csv
import glob
import os
import statistics
import sys

f = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True),
           key=os.path.getmtime)[-1]
ks = []
for r in csv.DictReader(open(f)):
    name = r.get("Kernel_Name", r.get("KernelName", ""))
    if "mmt::" not in name and "rocclr_copy" not in name:
        continue
    n = name.split("(")[0].replace("void ", "").replace("mmt::", "")
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), n))
ks.sort()
markers = {"ego": "k_flow_lm_split", "d3": "k_flow_lm<2>", "ransac": "k_pnp_hyp<5>"}
for chain, mk in markers.items():
    starts = [s for s, e, q, n in ks if n == mk]
    if len(starts) < 20:
        print(chain, "marker", mk, "seen", len(starts), "times: skipped")
        continue
    cut = len(starts) // 10
    t0, t1 = starts[cut], starts[-cut - 1]
    per = [b - a for a, b in zip(starts[cut:-cut - 1], starts[cut + 1:-cut])]
    q = [q for s, e, q, n in ks if n == mk][0]
    frames = len(per)
    dur = collections.defaultdict(int)
    busy = 0
    for s, e, qq, n in ks:
        if qq == q and t0 <= s < t1:
            dur[n] += e - s
            busy += e - s
    print("%s (queue %s): period median %.1f us, mean %.1f us over %d frames; busy %.1f%%" % (
        chain, q, statistics.median(per) / 1e3, statistics.mean(per) / 1e3, frames,
        100 * busy / (t1 - t0)))
    for n, d in sorted(dur.items(), key=lambda kv: -kv[1])[:12]:
        print("    %-24s %8.1f us per frame" % (n, d / frames / 1e3))

# interference: ego kernels' durations by what ran beside them on the other queues
ego_q = next((q for s, e, q, n in ks if n == "k_flow_lm_split"), None)
if ego_q is not None:
    others = [(s, e, n) for s, e, q, n in ks if q != ego_q and "copy" not in n]
    for target in ("k_pose_opt_l<2>", "k_match_fix", "k_flow_lm_split"):
        groups = collections.defaultdict(list)
        for s, e, q, n in ks:
            if n != target or q != ego_q:
                continue
            ov = collections.Counter()
            for s2, e2, n2 in others:
                o = min(e, e2) - max(s, s2)
                if o > 0:
                    ov[n2] += o
            key = "+".join(sorted(k for k, v in ov.items() if v > 0.2 * (e - s))) or "alone"
            groups[key].append((e - s) / 1e3)
        print(target)
        for k, v in sorted(groups.items(), key=lambda kv: -len(kv[1]))[:8]:
            print("    %-60s n=%4d mean %7.1f us" % (k[:60], len(v), statistics.mean(v)))
