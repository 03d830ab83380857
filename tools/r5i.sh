# Local BA change: LocalMapping GPU tests, then ba_bench timing and its kernel trace
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_localmap.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r5i_tests.log 2>&1 || { tail -40 gpurun_out/r5i_tests.log; exit 1; }
tail -3 gpurun_out/r5i_tests.log
MMT_BA_PROFILE=1 timeout -k 10 200 python tools/ba_bench.py --reps 64 > gpurun_out/r5i_ba.txt 2>&1 || { tail -20 gpurun_out/r5i_ba.txt; exit 1; }
tail -4 gpurun_out/r5i_ba.txt
rm -rf gpurun_out/r5i_trace
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r5i_trace -o run -- python tools/ba_bench.py --reps 8 > gpurun_out/r5i_trace.log 2>&1 || { tail -20 gpurun_out/r5i_trace.log; exit 1; }
python tools/rocpd_summary.py gpurun_out/r5i_trace | grep -E "kernel|ba2"
