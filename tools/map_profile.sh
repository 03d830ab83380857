# Host-side stage times of the map branch (MMT_MAP_PROFILE) and rocprofv3 kernel stats of a short
# C3 bench (argument: tag).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-map}
if [ -z "$SKIP_HOST" ]; then
MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --chunk 64 --no-cpu > gpurun_out/mapprof_$TAG.json 2> gpurun_out/mapprof_$TAG.err
grep "profile\]" gpurun_out/mapprof_$TAG.err
cat gpurun_out/mapprof_$TAG.json
fi
[ -n "$SKIP_RP" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 6 --warmup 1 --chunk 64 --no-cpu > gpurun_out/mapprof_rp_$TAG.json 2> gpurun_out/mapprof_rp_$TAG.err
cp "$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -print -quit)" gpurun_out/kstats_$TAG.csv
rm -rf gpurun_out/prof_$TAG
python - "$TAG" <<'PY'
import csv, sys
rows = list(csv.DictReader(open("gpurun_out/kstats_%s.csv" % sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    if r["Name"].startswith("void at::") or r["Name"].startswith("Cijk"):
        continue
    print("%-60s %8s %10.1f us avg %10.1f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
