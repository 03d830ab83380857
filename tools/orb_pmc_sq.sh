# SQ counters per ORB kernel (two separate --pmc passes over orb_microbench) plus the octree
# per-step cycle breakdown of the MMT_OCT_PROFILE build (tools/ab_build.sh octprof -DMMT_OCT_PROFILE).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-sq}
if [ -f multimot_track_amd/libmmt_octprof.so ]; then
  MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_octprof.so timeout -k 10 120 python tools/orb_microbench.py ${B:-64} 1 > gpurun_out/${tag}_octprof.log 2>&1
fi
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${tag}_p1 -o run -- python tools/orb_microbench.py ${B:-64} 3 > gpurun_out/${tag}_p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/${tag}_p2 -o run -- python tools/orb_microbench.py ${B:-64} 3 > gpurun_out/${tag}_p2.log 2>&1
{ python tools/pmc_summary.py gpurun_out/${tag}_p1; python tools/pmc_summary.py gpurun_out/${tag}_p2; } > gpurun_out/${tag}_summary.txt 2>&1 || true
