"""Print a window of a rocprofv3 kernel trace (kernel_trace.csv): start offset, duration, stream
(queue) and name of every kernel, to see how the tracker's chains overlap."""
import csv
import glob
import os
import sys

src = sys.argv[1]
tail_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
f = sorted(glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True),
           key=os.path.getmtime)[-1]
rows = list(csv.DictReader(open(f)))
ks = []
for r in rows:
    name = r.get("Kernel_Name", r.get("KernelName", ""))
    if "mmt::" not in name and "rocclr_copy" not in name:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    ks.append((s, e, q, name.split("(")[0].replace("void ", "")))
# memory copies (rocprofv3 --memory-copy-trace), shown as "copy <direction> <bytes>"
for fc in glob.glob(os.path.join(os.path.dirname(f), "*memory_copy_trace.csv")):
    for r in csv.DictReader(open(fc)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ks.append((s, e, "cp", "copy %s %s B" % (r.get("Direction", "?"), r.get("Size", "?"))))
ks.sort()
end = max(k[1] for k in ks)
t0 = end - tail_ms * 1e6
busy = {}
for s, e, q, n in ks:
    if s < t0:
        continue
    busy[q] = busy.get(q, 0) + (e - s)
    print("%9.1f us  %8.1f us  q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, q, n))
print("busy per queue (us):", {k: round(v / 1e3, 1) for k, v in busy.items()})
