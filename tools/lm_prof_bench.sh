# LM phase clocks (MMT_LM_PROFILE build: tools/ab_build.sh lmprof --src mmt_lm.hip -DMMT_LM_PROFILE)
# on the bench's own solves and on the object-like probe.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_lmprof.so
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/lmprof_bench.log 2>&1
grep -c lmprof gpurun_out/lmprof_bench.log
timeout -k 10 100 python tools/lm_trial_bench.py 208 3 > gpurun_out/lmprof_probe.log 2>&1
tail -3 gpurun_out/lmprof_probe.log
