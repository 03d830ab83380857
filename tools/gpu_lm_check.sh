# The flow-solve (D2/D3) probe tests and the tracking tests, then the bench line.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_track.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_lm1.log 2>&1 || { tail -60 gpurun_out/gpu_lm1.log; exit 1; }
tail -3 gpurun_out/gpu_lm1.log
timeout -k 10 400 python bench.py > gpurun_out/bench_${1:-lm}.json 2> gpurun_out/bench_${1:-lm}.err
cat gpurun_out/bench_${1:-lm}.json
