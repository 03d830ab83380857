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
rows = list(csv.DictReader(open(files[-1])))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[name].add(r["Dispatch_Id"])
for name, cs in sorted(acc.items()):
    nd = max(len(disp[name]), 1)
    print("%-32s n=%-4d %s" % (name, nd, " ".join("%s=%.4g" % (k, v / nd) for k, v in sorted(cs.items()))))
