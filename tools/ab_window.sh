# A/B of ORB builds: window time (tracker context) and standalone kernel times (MMT_ORB_SCHED=2)
# at batch B (default 64) for the default libmmt.so and each libmmt_<sfx>.so named.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base "$@"; do
  if [ "$v" = base ]; then unset MMT_LIB_PATH; else export MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_$v.so; fi
  echo "== $v window: $(timeout -k 10 120 python tools/orb_window_bench.py ${B:-64} 20 2>&1 | grep batch=)"
  rm -rf gpurun_out/abw_$v
  MMT_ORB_SCHED=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abw_$v -o run -- python tools/orb_microbench.py ${B:-64} 10 > gpurun_out/abw_$v.log 2>&1
  python tools/rocprof_summary.py gpurun_out/abw_$v gpurun_out/abw_${v}_stats.csv | grep mmt:: || true
  rm -rf gpurun_out/abw_$v
done
