# ORB change round trip: ORB + tracking parity tests, window and per-kernel times (schedule 0),
# octree phase clocks (profiling build libmmt_octprof.so: tools/ab_build.sh octprof -DMMT_OCT_PROFILE)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_track.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orb_tests.log 2>&1 || { tail -30 gpurun_out/orb_tests.log; exit 1; }
tail -1 gpurun_out/orb_tests.log
bash tools/orb_sched.sh 0
if [ -f multimot_track_amd/libmmt_octprof.so ]; then
  MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_octprof.so timeout -k 10 120 python tools/orb_microbench.py 32 2 > gpurun_out/octprof.log 2>&1
  grep -E "octprof|steps" gpurun_out/octprof.log | tail -10
fi
