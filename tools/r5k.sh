# k_pyramid: ORB bit-exact tests, window A/B against the k_resize chain, standalone kernel times
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r5k_tests.log 2>&1 || { tail -40 gpurun_out/r5k_tests.log; exit 1; }
tail -2 gpurun_out/r5k_tests.log
for v in 1 0 1 0; do
  MMT_PYR=$v timeout -k 10 120 python tools/orb_window_bench.py 128 20 > gpurun_out/r5k_pyr$v.log 2>&1 || { tail -20 gpurun_out/r5k_pyr$v.log; exit 1; }
  echo "pyr=$v $(grep window gpurun_out/r5k_pyr$v.log)"
done
for v in 1 0; do
  MMT_PYR=$v timeout -k 10 120 python tools/orb_window_bench.py 1 200 > gpurun_out/r5k_b1_pyr$v.log 2>&1 || { tail -20 gpurun_out/r5k_b1_pyr$v.log; exit 1; }
  echo "batch1 pyr=$v $(grep window gpurun_out/r5k_b1_pyr$v.log)"
done
rm -rf gpurun_out/r5k_orbk
MMT_ORB_SCHED=2 timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/r5k_orbk -o run -- python tools/orb_window_bench.py 128 5 > gpurun_out/r5k_orbk.log 2>&1 || { tail -20 gpurun_out/r5k_orbk.log; exit 1; }
grep window gpurun_out/r5k_orbk.log
python tools/rocpd_summary.py gpurun_out/r5k_orbk --by-grid | grep -E "kernel|k_blur|k_resize|k_pyramid|k_octree|k_orient|k_gray|k_fast"
