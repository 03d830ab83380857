set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/orb_sched.sh 2 0
MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_octprof.so timeout -k 10 120 python tools/orb_microbench.py 32 2 > gpurun_out/octprof.log 2>&1
grep -c octprof gpurun_out/octprof.log
