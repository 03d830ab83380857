set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r02a.json 2> gpurun_out/bench_r02a.err
cat gpurun_out/bench_r02a.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --seqs-per-gpu 4 --no-cpu > gpurun_out/bench_r02a_k4.json 2> gpurun_out/bench_r02a_k4.err
cat gpurun_out/bench_r02a_k4.json
rm -rf gpurun_out/benchk
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/benchk -o run -- python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/benchk.log 2>&1
python tools/rocprof_summary.py gpurun_out/benchk gpurun_out/bench_r02a_kernel_stats.csv | grep "mmt::" | head -30
rm -rf gpurun_out/benchk
