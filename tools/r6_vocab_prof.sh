# Kernel trace of the vocabulary bench (short) and the BA host phases (MMT_BA_PROFILE=1).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-vp}
common="--steps 4 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0"
MMT_BA_PROFILE=1 timeout -k 10 300 python bench.py $common > gpurun_out/${tag}_ba.json 2> gpurun_out/${tag}_ba.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_kt -o run -- python bench.py $common > gpurun_out/${tag}_kt.json 2> gpurun_out/${tag}_kt.err
f=$(find gpurun_out/${tag}_kt -name "*kernel_stats.csv" | head -1)
head -25 $f | cut -d, -f1-8
grep -h "ba prof\|BA prof\|\[mmt ba" gpurun_out/${tag}_ba.err | tail -5
