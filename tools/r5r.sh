# The bench command under rocprofv3 --kernel-trace --stats (csv): the kernel_stats summary and the
# ORB window spans (k_gray_depth start to the last ORB kernel's end) from the trace, for profiles/
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/r5r
( for i in $(seq 1 15); do sleep 50; echo "heartbeat $i"; done ) &
hb=$!
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5r -o run -- python bench.py --no-cpu --single-frames 0 > gpurun_out/r5r_bench.json 2> gpurun_out/r5r_bench.err || { kill $hb; tail -20 gpurun_out/r5r_bench.err; exit 1; }
cp "$(find /tmp/r5r -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5r_kernel_stats.csv
f=$(find /tmp/r5r -name '*kernel_trace.csv' -print -quit)
grep -E "k_gray_depth|k_resize|k_pyramid|k_fast|k_octree|k_blur|k_orient_desc" "$f" > /tmp/r5r_orb.csv || true
head -1 "$f" > gpurun_out/r5r_trace_header.csv
python - /tmp/r5r_orb.csv gpurun_out/r5r_trace_header.csv <<'PY' > gpurun_out/r5r_windows.txt
import csv, sys
hdr = next(csv.reader(open(sys.argv[2])))
rows = []
for r in csv.reader(open(sys.argv[1])):
    d = dict(zip(hdr, r))
    rows.append((int(d["Start_Timestamp"]), int(d["End_Timestamp"]), d["Kernel_Name"], int(d.get("Grid_Size_Y", d.get("Grid_Y", "1")) or 1)))
rows.sort()
spans, t0, end = [], None, 0
for st, en, nm, gy in rows:
    if "k_gray_depth" in nm and gy == 128:
        if t0 is not None:
            spans.append((end - t0) / 1e3)
        t0, end = st, en
    elif t0 is not None:
        end = max(end, en)
if t0 is not None:
    spans.append((end - t0) / 1e3)
sp = sorted(spans)
print("ORB windows at batch 128 in the bench (k_gray_depth start to the last ORB kernel end): %d, mean %.1f us, median %.1f us, min %.1f us" % (len(sp), sum(sp) / len(sp), sp[len(sp) // 2], sp[0]))
PY
kill $hb || true
rm -rf /tmp/r5r /tmp/r5r_orb.csv
cat gpurun_out/r5r_windows.txt
