set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_track.py -m gpu -x -v --timeout 240 --timeout-method thread -k "c3_long or lost_frame" > gpurun_out/r5a_c3long.log 2>&1 || { tail -40 gpurun_out/r5a_c3long.log; exit 1; }
tail -3 gpurun_out/r5a_c3long.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r5a_suite.log 2>&1 || { tail -40 gpurun_out/r5a_suite.log; exit 1; }
tail -3 gpurun_out/r5a_suite.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || { tail -20 gpurun_out/r5a_bench.err; exit 1; }
cat gpurun_out/r5a_bench.json
