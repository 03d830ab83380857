# Fuse host loops: map parity tests, then A/B against the previous build (libmmt_prof.so)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_localmap.py tests/test_gpu_track.py -m gpu -x -v --timeout 240 --timeout-method thread -k "localmap or map_graph or culling or c3_long or lost_frame" > gpurun_out/r5s_tests.log 2>&1 || { tail -40 gpurun_out/r5s_tests.log; exit 1; }
tail -2 gpurun_out/r5s_tests.log
bash tools/r5o.sh
