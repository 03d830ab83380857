# ORB tests and the batch-128 window traffic with the default XCD order
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r5v_tests.log 2>&1 || { tail -40 gpurun_out/r5v_tests.log; exit 1; }
tail -1 gpurun_out/r5v_tests.log
timeout -k 10 400 bash tools/orb_traffic.sh 128 > gpurun_out/r5v_orbt.log 2>&1 || { tail -20 gpurun_out/r5v_orbt.log; exit 1; }
cat gpurun_out/r5v_orbt.log
