# HBM traffic of the batched ORB launch sequence: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes over the tracker's ORB window (tools/orb_window_bench.py: batch B,
# 1 warm-up + 3 timed chunks).  Usage: orb_traffic.sh [B=64]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${1:-64}
rm -rf gpurun_out/orbf gpurun_out/orbw
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/orbf -o run -- python tools/orb_window_bench.py $B 3 > gpurun_out/orbf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/orbw -o run -- python tools/orb_window_bench.py $B 3 > gpurun_out/orbw.log 2>&1
python tools/traffic_from_pmc.py gpurun_out/orbf gpurun_out/orbw 4 1242x375_n2000_b$B gpurun_out/traffic.json | tee gpurun_out/orb_traffic.txt
rm -rf gpurun_out/orbf gpurun_out/orbw
