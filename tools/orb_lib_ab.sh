# Standalone ORB kernel times (one stream, batch B) of libmmt.so against libmmt_prof.so.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libmmt.so libmmt_prof.so; do
  rm -rf gpurun_out/lab
  MMT_LIB_PATH=$PWD/multimot_track_amd/$lib MMT_ORB_SCHED=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lab -o run -- python tools/orb_microbench.py ${B:-128} 20 > gpurun_out/lab.log 2>&1
  echo "== $lib"
  python tools/rocprof_summary.py gpurun_out/lab gpurun_out/lab_stats.csv | grep mmt:: || true
  echo "window: $(MMT_LIB_PATH=$PWD/multimot_track_amd/$lib timeout -k 10 120 python tools/orb_window_bench.py ${B:-128} 20 2>&1 | grep batch=)"
done
rm -rf gpurun_out/lab
