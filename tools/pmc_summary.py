"""Sum rocprofv3 --pmc counter_collection.csv per kernel: prints kernel, dispatches and the mean
value per dispatch of every counter collected."""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
files = sorted(glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True),
               key=os.path.getmtime)
if files:
    recs = [(r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), r["Dispatch_Id"])
            for r in csv.DictReader(open(files[-1]))]
else:  # rocprofv3 writing a results database
    import sqlite3
    db = sorted(glob.glob(os.path.join(src, "**", "*.db"), recursive=True),
                key=os.path.getmtime)[-1]
    recs = list(sqlite3.connect(db).execute(
        "select kernel_name, counter_name, value, dispatch_id from counters_collection"))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for kn, cn, val, did in recs:
    name = kn.split("(")[0].replace("void ", "")
    acc[name][cn] += float(val)
    disp[name].add(did)
for name, cs in sorted(acc.items()):
    nd = max(len(disp[name]), 1)
    print("%-32s n=%-4d %s" % (name, nd, " ".join("%s=%.4g" % (k, v / nd) for k, v in sorted(cs.items()))))
