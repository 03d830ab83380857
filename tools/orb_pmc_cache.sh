# Cache-side counters per ORB kernel (separate --pmc passes over orb_microbench).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d gpurun_out/pc1 -o run -- python tools/orb_microbench.py 32 2 > gpurun_out/pc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum --output-format csv -d gpurun_out/pc2 -o run -- python tools/orb_microbench.py 32 2 > gpurun_out/pc2.log 2>&1 || true
python tools/pmc_summary.py gpurun_out/pc1 | grep mmt::
python tools/pmc_summary.py gpurun_out/pc2 | grep mmt:: || tail -5 gpurun_out/pc2.log
