# C4 / C5 depth: the 400-frame C4 and 250-frame C5 parity tests
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py -m gpu -x -v -s --timeout 400 --timeout-method thread -k "400_frames or 250_frames" > gpurun_out/r5j_tests.log 2>&1 || { tail -40 gpurun_out/r5j_tests.log; exit 1; }
grep -E "frames'|PASSED|passed|failed" gpurun_out/r5j_tests.log | tail -8
