# Two SQ counter passes over the ORB microbench (one rocprofv3 --pmc run each).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/orbp1 gpurun_out/orbp2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/orbp1 -o run -- python tools/orb_microbench.py 32 3 > gpurun_out/orbp1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD -d gpurun_out/orbp2 -o run -- python tools/orb_microbench.py 32 3 > gpurun_out/orbp2.log 2>&1
python tools/pmc_summary.py gpurun_out/orbp1 | grep mmt
python tools/pmc_summary.py gpurun_out/orbp2 | grep mmt
