set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
MMT_ORB_VERBOSE=1 timeout -k 10 60 python tools/orb_microbench.py 32 2 2>&1 | grep -v amdgpu.ids
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pp1 -o run -- python tools/orb_microbench.py 32 2 > gpurun_out/pp1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pp2 -o run -- python tools/orb_microbench.py 32 2 > gpurun_out/pp2.log 2>&1
python tools/pmc_summary.py gpurun_out/pp1 | grep mmt::
python tools/pmc_summary.py gpurun_out/pp2 | grep mmt::
