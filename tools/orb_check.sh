# ORB round trip: parity tests, window time under both launch schedules, per-kernel dispatch times.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orb_tests.log 2>&1 || { tail -30 gpurun_out/orb_tests.log; exit 1; }
tail -1 gpurun_out/orb_tests.log
for s in 0 1; do
  echo "sched $s: $(MMT_ORB_SCHED=$s timeout -k 10 120 python tools/orb_microbench.py 32 20 2>&1 | tail -1)"
  echo "sched $s window: $(MMT_ORB_SCHED=$s timeout -k 10 120 python tools/orb_window_bench.py 32 20 2>&1 | grep batch=)"
done
rm -rf gpurun_out/orbk
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/orbk -o run -- python tools/orb_microbench.py 32 20 > gpurun_out/orbk.log 2>&1
python tools/dispatch_times.py gpurun_out/orbk/run_results.db
