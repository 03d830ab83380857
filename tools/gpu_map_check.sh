set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_track.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_map1.log 2>&1 || { tail -60 gpurun_out/gpu_map1.log; exit 1; }
tail -5 gpurun_out/gpu_map1.log
