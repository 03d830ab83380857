"""Per-frame kernel timeline of a filtered rocprofv3 kernel trace (columns Kernel_Name, Queue_Id,
Start_Timestamp, End_Timestamp, as tools/one_frame_bench.py under `rocprofv3 --kernel-trace`):
frames are cut at every launch of the kernel named by MMT_CUT (default `k_gray_depth`, one per
call in the one-frame pattern; `k_static_samples` cuts the frames of a chunked run).  Prints, for
the frames asked, each kernel's start offset, duration, the idle gap before it on its queue and
its name; and over all frames the device time and launch count per kernel name per frame, and
the busy fraction of the frame's wall time.
Usage: frame_timeline.py trace.csv [frame numbers to list, e.g. 30 31]"""
import collections
import csv
import os
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
show = {int(x) for x in sys.argv[2:]}
ks = []
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mmt::", "")
    name = name.replace("(anonymous namespace)::", "")
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], name))
ks.sort()
cut = os.environ.get("MMT_CUT", "k_gray_depth")
cuts = [i for i, k in enumerate(ks) if k[3].startswith(cut)]
tot = collections.defaultdict(float)
cnt = collections.defaultdict(int)
walls, busy = [], []
for fi in range(len(cuts) - 1):
    seg = ks[cuts[fi]:cuts[fi + 1]]
    t0, t1 = seg[0][0], ks[cuts[fi + 1]][0]
    walls.append((t1 - t0) / 1e3)
    # union of busy intervals
    iv = sorted((s, e) for s, e, _, _ in seg)
    b, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            b += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    b += ce - cs
    busy.append(b / 1e3)
    for s, e, q, n in seg:
        tot[n] += (e - s) / 1e3
        cnt[n] += 1
    if fi in show:
        print("---- frame %d: wall %.1f us, device busy %.1f us" % (fi, walls[-1], busy[-1]))
        last = {}
        for s, e, q, n in seg:
            gap = (s - last[q]) / 1e3 if q in last else 0.0
            last[q] = e
            print("%9.1f %8.1f  gap %7.1f  q%s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, q, n))
nf = len(walls)
print("%d frames: wall %.1f us per frame, device busy %.1f us per frame" %
      (nf, sum(walls) / nf, sum(busy) / nf))
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:40]:
    print("%-40s %6.2f launches %8.1f us per frame" % (n[:40], cnt[n] / nf, t / nf))
