# ORB bit-exact GPU tests, then the standalone kernel times (one stream) and the tracker's window
# at batch B (default 128).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 240 2>&1 | tail -2
B=${B:-128} bash tools/orb_sched.sh 2 0
