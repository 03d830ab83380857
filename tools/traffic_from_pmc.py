"""HBM traffic of one batched ORB launch sequence from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950), for profiles/traffic.json (bench.py roofline.traffic).

Usage: traffic_from_pmc.py <fetch_dir> <write_dir> <launches> <key> [json_out]
Counter values are KB per dispatch (rocprofv3).  The guide's x2 FETCH_SIZE correction is for
16-byte-per-lane streaming reads; the ORB kernels read 1-4 bytes per lane, so it is not applied
(the calibration against k_resize's known read bytes is printed instead)."""
import collections
import csv
import glob
import json
import os
import sys

ORB = ("k_resize", "k_fast", "k_octree", "k_blur", "k_orient_desc")


def load(d, counter):
    files = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True),
                   key=os.path.getmtime)
    if files:
        recs = [(r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), r["Dispatch_Id"])
                for r in csv.DictReader(open(files[-1]))]
    else:  # rocprofv3 writing a results database
        import sqlite3
        db = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True),
                    key=os.path.getmtime)[-1]
        recs = list(sqlite3.connect(db).execute(
            "select kernel_name, counter_name, value, dispatch_id from counters_collection"))
    tot = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for kn, cn, val, did in recs:
        if cn != counter:
            continue
        # "void mmt::k_fast<40>(...)" -> "k_fast"
        name = kn.split("(")[0].replace("void ", "").replace("mmt::", "").split("<")[0]
        tot[name] += float(val)
        n[name].add(did)
    return tot, n


fd, wd, launches, key = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
out = sys.argv[5] if len(sys.argv) > 5 else None
fetch, nf = load(fd, "FETCH_SIZE")
write, nw = load(wd, "WRITE_SIZE")
total = 0.0
print("kernel            dispatches  FETCH_KB/launch  WRITE_KB/launch")
for k in ORB:
    fk = fetch.get(k, 0.0) / launches
    wk = write.get(k, 0.0) / launches
    total += (fk + wk) * 1024
    print("%-16s %10d %16.1f %16.1f" % (k, len(nf.get(k, ())), fk, wk))
print("ORB launch sequence traffic: %.0f bytes (%.1f MB)" % (total, total / 1e6))
if out:
    d = {}
    if os.path.exists(out):
        d = json.load(open(out))
    d[key] = int(total)
    d["_note"] = ("HBM-side bytes (rocprofv3 FETCH_SIZE + WRITE_SIZE, separate passes, KB -> B) "
                  "summed over the ORB kernels of one batched launch sequence; see DESIGN.md")
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
