# ORB kernel times under each launch schedule (MMT_ORB_SCHED: bit 0 fused pyramid, bit 1 one
# stream = standalone kernel durations).  Usage (GPU box): bash tools/orb_sched.sh [scheds]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in ${@:-0 1 2 3}; do
  rm -rf gpurun_out/sched_$s
  MMT_ORB_SCHED=$s timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sched_$s -o run -- python tools/orb_microbench.py ${B:-64} 20 > gpurun_out/sched_$s.log 2>&1
  echo "== sched $s: $(grep batch= gpurun_out/sched_$s.log)"
  python tools/rocprof_summary.py gpurun_out/sched_$s gpurun_out/sched_${s}_stats.csv | grep mmt:: || true
  echo "window: $(MMT_ORB_SCHED=$s timeout -k 10 120 python tools/orb_window_bench.py ${B:-64} 20 2>&1 | grep batch=)"
done
