# ORB round trip on the GPU box: parity tests, then the window and per-kernel times.
# Usage: bash tools/orb_quick.sh [tag]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
bash tools/orb_trace.sh $tag
python tools/rocprof_summary.py gpurun_out/$tag gpurun_out/${tag}_stats.csv | grep mmt:: || true
