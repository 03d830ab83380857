# Kernel trace of the standalone ORB launch sequence (orb_microbench) and of the tracker's ORB
# window (orb_window_bench): per-kernel stats plus a timeline of the last launch.
# Usage (GPU box): bash tools/orb_trace.sh [tag]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=${1:-orbt}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/orb_window_bench.py ${B:-64} 20 > gpurun_out/${tag}_window.log 2>&1
timeout -k 10 120 python tools/orb_microbench.py ${B:-64} 20 > gpurun_out/${tag}_micro.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag} -o run -- python tools/orb_microbench.py ${B:-64} 20 > gpurun_out/${tag}_prof.log 2>&1
python tools/timeline.py gpurun_out/${tag} 0.5 > gpurun_out/${tag}_timeline.txt
cat gpurun_out/${tag}_window.log gpurun_out/${tag}_micro.log
