# ORB window (tracker context, kitti_sample frames) at batch 128 for MMT_ORB_PARTS = 1, 2, 4, then
# the bit-exact ORB GPU tests under the default.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for p in ${PARTS:-1 2 4}; do
  echo "parts=$p $(MMT_ORB_PARTS=$p timeout -k 10 120 python tools/orb_window_bench.py ${B:-128} 10 2>&1 | tail -1)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 240 2>&1 | tail -2
