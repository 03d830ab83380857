# Per-phase cycle counts of k_fast (MMT_FAST_PROFILE build: tools/ab_build.sh fprof
# -DMMT_FAST_PROFILE) on the ORB microbench.  Usage (GPU box): bash tools/fast_prof.sh
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_fprof.so
timeout -k 10 60 python tools/orb_microbench.py 32 1 > gpurun_out/fastprof.log 2>&1
grep fastprof gpurun_out/fastprof.log | sort -t' ' -k3 -n | head -40
