# SQ instruction counters of the ORB window kernels (one rocprofv3 --pmc pass).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/orbsq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/orbsq -o run -- python tools/orb_window_bench.py 32 3 > gpurun_out/orbsq.log 2>&1
python tools/pmc_summary.py gpurun_out/orbsq | grep "k_gray\|k_resize\|k_fast\|k_octree\|k_blur\|k_orient" | tee gpurun_out/orb_sq.txt
rm -rf gpurun_out/orbsq
