# XCD-contiguous blur / resize: ORB bit-exact tests, the window at batch 128, HBM traffic
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r5t_tests.log 2>&1 || { tail -40 gpurun_out/r5t_tests.log; exit 1; }
tail -1 gpurun_out/r5t_tests.log
for r in 1 2 3; do
  timeout -k 10 120 python tools/orb_window_bench.py 128 20 > gpurun_out/r5t_w.log 2>&1 || { tail -20 gpurun_out/r5t_w.log; exit 1; }
  grep window gpurun_out/r5t_w.log
done
timeout -k 10 400 bash tools/orb_traffic.sh 128 > gpurun_out/r5t_orbt.log 2>&1 || { tail -20 gpurun_out/r5t_orbt.log; exit 1; }
cat gpurun_out/r5t_orbt.log
