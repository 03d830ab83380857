# kernel timeline of the local BA chain (ba_bench under rocprofv3 --kernel-trace)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/ba_trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ba_trace -o run -- python tools/ba_bench.py --reps 8 > gpurun_out/r5f_ba.txt 2>&1
f=$(find gpurun_out/ba_trace -name '*kernel_trace.csv' -print -quit)
python - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "ba2" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last solve: from the last k_ba2_init
idx = [i for i, r in enumerate(rows) if "ba2_init" in r["Kernel_Name"]]
seg = rows[idx[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
prev = None
for r in seg[:60]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    name = r["Kernel_Name"].split("(")[0].split("::")[-1]
    print("%8.1f  dur %6.1f  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, name))
    prev = e
print("total", (int(seg[-1]["End_Timestamp"]) - t0) / 1e3, "us for", len(seg), "kernels")
PY
