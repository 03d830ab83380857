# Host-side LocalMapping changes: map / tracking parity tests, then the host stage profile
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_localmap.py tests/test_gpu_track.py -m gpu -x -v --timeout 240 --timeout-method thread -k "localmap or map_graph or culling or local_ba or c3_long or lost_frame" > gpurun_out/r5m_tests.log 2>&1 || { tail -40 gpurun_out/r5m_tests.log; exit 1; }
tail -2 gpurun_out/r5m_tests.log
MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --chunk 64 --no-cpu --single-frames 0 > gpurun_out/r5m_prof.json 2> gpurun_out/r5m_prof.err
grep "profile\]" gpurun_out/r5m_prof.err | head -6
