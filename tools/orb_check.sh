set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orb_tests.log 2>&1 || { tail -30 gpurun_out/orb_tests.log; exit 1; }
tail -1 gpurun_out/orb_tests.log
if [ -f multimot_track_amd/libmmt_octprof.so ]; then MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_octprof.so timeout -k 10 120 python tools/orb_microbench.py 1 1 2>&1 | grep "steps\|level=0 \|level=442" | head -3; fi
timeout -k 10 120 python tools/orb_microbench.py 32 20 2>&1 | tail -1
rm -rf gpurun_out/orbk
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/orbk -o run -- python tools/orb_microbench.py 32 20 > gpurun_out/orbk.log 2>&1
python tools/dispatch_times.py gpurun_out/orbk/run_results.db
