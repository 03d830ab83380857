"""HBM traffic of one batched ORB window (k_gray_depth + the ORB launch sequence) from two
rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), for
profiles/traffic.json (bench.py roofline.traffic).

Usage: traffic_from_pmc.py <fetch_dir> <write_dir> <launches> <key> [json_out]
Counter values are KB per dispatch (rocprofv3), KB = 1024 B.  gfx950 correction
(MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of coalesced streaming reads, so it
is doubled; calibrated here on k_gray_depth, whose reads are known exactly (5 B per pixel: BGR +
u16 disparity, read once), and printed.  WRITE_SIZE is taken as is (k_gray_depth's known 5 B per
pixel of writes calibrate it too)."""
import collections
import csv
import glob
import json
import os
import sys

ORB = ("k_gray_depth", "k_resize", "k_fast", "k_octree", "k_blur", "k_orient_desc")


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
raw = 0.0
for k in ORB:
    fk = fetch.get(k, 0.0) / launches
    wk = write.get(k, 0.0) / launches
    raw += (fk + wk) * 1024
    total += (2 * fk + wk) * 1024
    print("%-16s %10d %16.1f %16.1f" % (k, len(nf.get(k, ())), fk, wk))
W, H = 1242, 375
B = int(key.rsplit('_b', 1)[1])  # key 1242x375_n2000_b<batch>
known = 5.0 * W * H * B
print("calibration k_gray_depth: known reads %.1f MB, FETCH_SIZE %.1f MB (x%.2f); known writes "
      "%.1f MB, WRITE_SIZE %.1f MB" % (known / 1e6, fetch.get("k_gray_depth", 0) / launches *
                                       1024 / 1e6, known / max(fetch.get("k_gray_depth", 0) /
                                                               launches * 1024, 1),
                                       known / 1e6, write.get("k_gray_depth", 0) / launches *
                                       1024 / 1e6))
print("ORB window traffic: raw FETCH+WRITE %.1f MB; corrected 2*FETCH+WRITE %.0f bytes (%.1f MB)"
      % (raw / 1e6, total, total / 1e6))
if out:
    d = {}
    if os.path.exists(out):
        d = json.load(open(out))
    d[key] = int(total)
    d["_note"] = ("HBM-side bytes (rocprofv3 2 x FETCH_SIZE + WRITE_SIZE, separate passes, KB -> B, "
                  "gfx950 FETCH correction calibrated on k_gray_depth) "
                  "summed over the kernels of one batched ORB window (k_gray_depth + the ORB "
                  "launch sequence; tools/orb_traffic.sh); see DESIGN.md")
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
