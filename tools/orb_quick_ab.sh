set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_track.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orb_tests.log 2>&1 || { tail -30 gpurun_out/orb_tests.log; exit 1; }
tail -1 gpurun_out/orb_tests.log
bash tools/ab_window.sh "$@"
