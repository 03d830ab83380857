# BA change: LocalMapping GPU tests, the long C3 test, then ba_bench timing
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_localmap.py tests/test_gpu_track.py -m gpu -x -v --timeout 240 --timeout-method thread -k "local_ba or localmap or map_graph or c3_long or lost_frame" > gpurun_out/r5e_tests.log 2>&1 || { tail -40 gpurun_out/r5e_tests.log; exit 1; }
tail -3 gpurun_out/r5e_tests.log
MMT_BA_PROFILE=1 timeout -k 10 200 python tools/ba_bench.py --reps 64 > gpurun_out/r5e_ba.txt 2>&1 || { tail -20 gpurun_out/r5e_ba.txt; exit 1; }
tail -6 gpurun_out/r5e_ba.txt
