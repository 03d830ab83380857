# MMT_ORB_XCD A/B: window at batch 128 per setting, interleaved
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for x in 0 1 2 3; do
    MMT_ORB_XCD=$x timeout -k 10 120 python tools/orb_window_bench.py 128 30 > gpurun_out/r5u.log 2>&1 || { tail -20 gpurun_out/r5u.log; exit 1; }
    echo "xcd=$x $(grep window gpurun_out/r5u.log)"
  done
done
