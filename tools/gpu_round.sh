# One GPU round trip: the -m gpu parity suite, then the driver's bench command (argument: tag).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
