# Round 5: full GPU suite, the local BA bench, and the driver's default bench line
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r5h_suite.log 2>&1 || { tail -40 gpurun_out/r5h_suite.log; exit 1; }
tail -3 gpurun_out/r5h_suite.log
MMT_BA_PROFILE=1 timeout -k 10 200 python tools/ba_bench.py --reps 64 > gpurun_out/r5h_ba.txt 2>&1 || { tail -20 gpurun_out/r5h_ba.txt; exit 1; }
tail -4 gpurun_out/r5h_ba.txt
timeout -k 10 600 python bench.py > gpurun_out/r5h_bench.json 2> gpurun_out/r5h_bench.err || { tail -20 gpurun_out/r5h_bench.err; exit 1; }
cat gpurun_out/r5h_bench.json
