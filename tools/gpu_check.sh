# GPU round trip used during development: parity tests, ORB microbench, ORB kernel stats.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python tools/orb_microbench.py 32 20 > gpurun_out/orb_mb.log 2>&1
cat gpurun_out/orb_mb.log | tail -1
rm -rf gpurun_out/orbk
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/orbk -o run -- python tools/orb_microbench.py 32 20 > gpurun_out/orbk.log 2>&1
python tools/rocprof_summary.py gpurun_out/orbk gpurun_out/orbk_stats.csv | grep "mmt::\|copy"
