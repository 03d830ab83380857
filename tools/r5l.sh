# k_pyramid against the k_resize chain by batch size (window per batch, tools/orb_window_bench.py)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 1 4 16 32 64; do
  for m in 0 1000; do
    MMT_PYR_MAX_FRAMES=$m timeout -k 10 120 python tools/orb_window_bench.py $b 50 > gpurun_out/r5l.log 2>&1 || { tail -20 gpurun_out/r5l.log; exit 1; }
    echo "batch=$b pyr_max_frames=$m $(grep window gpurun_out/r5l.log)"
  done
done
