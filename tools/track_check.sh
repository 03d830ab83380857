# Tracker change check: the GPU tracking/C-ABI tests, then the driver's bench line.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_${1:-chk}.json 2> gpurun_out/bench_${1:-chk}.err
cat gpurun_out/bench_${1:-chk}.json
