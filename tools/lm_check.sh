# LM change round trip: flow-solve + tracking parity tests, LM phase clocks on the bench's solves
# (profiling build libmmt_lmprof.so), then the bench line.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_lmprof.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/lmprof_bench.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_lm.json 2> gpurun_out/bench_lm.err
cat gpurun_out/bench_lm.json
