# Pose-opt variants launched widest first (MMT_PO_WIDE_FIRST): tracking + pose-opt parity, in-box
# bench A/B, then a short kernel trace for the motion-model solve's k_pose_opt_l<4> durations
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_localmap.py -m gpu -x -q --timeout 240 --timeout-method thread -k "pose or c3_long or lost_frame or synthetic or split or contexts or culling" > gpurun_out/r5zd_tests.log 2>&1 || { tail -30 gpurun_out/r5zd_tests.log; exit 1; }
tail -1 gpurun_out/r5zd_tests.log
for v in 1 0 1 0 1 0; do
  MMT_PO_WIDE_FIRST=$v timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --single-frames 128 --c2-steps 2 > gpurun_out/r5zd_$v.json 2> gpurun_out/r5zd_$v.err
  echo "== wide_first=$v $(python -c "import json;d=json.loads(open('gpurun_out/r5zd_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['c2']['value'], d['config']['one_frame_per_call']['ms_per_frame'], d['valid'])")"
done
rm -rf /tmp/etr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/etr -o run -- python bench.py --steps 3 --warmup 1 --chunk 64 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/r5zd_trace.log 2>&1
f="$(find /tmp/etr -name '*kernel_trace.csv' -print -quit)"
python - "$f" <<'PY'
import csv, sys, statistics as S
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
cuts = [i for i, k in enumerate(ks) if k[3].startswith("mmt::k_flow_lm_split")]
v = {}
for fi in range(max(0, len(cuts) - 129), len(cuts) - 1):
    q = ks[cuts[fi]][2]
    po = [k for k in ks[cuts[fi]:cuts[fi + 1]] if k[2] == q and "k_pose_opt_l" in k[3]]
    for j, k in enumerate(po):
        v.setdefault((j, k[3].split("(")[0]), []).append((k[1] - k[0]) / 1e3)
for key, d in sorted(v.items()):
    d.sort()
    print(key, len(d), "median %.1f p90 %.1f max %.1f" % (S.median(d), d[int(0.9 * len(d))], d[-1]))
walls = [(ks[cuts[i + 1]][0] - ks[cuts[i]][0]) / 1e3 for i in range(max(0, len(cuts) - 129), len(cuts) - 1)]
print("frame wall median %.1f us" % S.median(walls))
PY
