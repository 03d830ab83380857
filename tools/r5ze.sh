# Local BA LDL^T two columns per step: BA + LocalMapping + tracking parity, ba_bench timing
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_localmap.py tests/test_gpu_track.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c4 and not c5" > gpurun_out/r5ze_tests.log 2>&1 || { tail -30 gpurun_out/r5ze_tests.log; exit 1; }
tail -1 gpurun_out/r5ze_tests.log
MMT_BA_PROFILE=1 timeout -k 10 200 python tools/ba_bench.py > gpurun_out/r5ze_ba_bench.txt 2>&1
grep -v amdgpu.ids gpurun_out/r5ze_ba_bench.txt | tail -6
MMT_BA_PROFILE=1 timeout -k 10 200 python tools/ba_bench.py --kfs 16 > gpurun_out/r5ze_ba_bench16.txt 2>&1
grep -v amdgpu.ids gpurun_out/r5ze_ba_bench16.txt | tail -3
