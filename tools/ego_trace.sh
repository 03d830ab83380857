# Kernel + memory-copy timeline of the last few ms of a short C3 bench (the ego chain's gaps).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/etr
timeout -k 10 300 rocprofv3 --kernel-trace ${ETR_EXTRA} --output-format csv -d gpurun_out/etr -o run -- python bench.py --steps 3 --warmup 1 --chunk 64 --no-cpu ${BENCH_EXTRA} > gpurun_out/etr.log 2>&1
python tools/timeline.py gpurun_out/etr ${TAIL_MS:-4} > gpurun_out/ego_timeline.txt
python tools/queue_busy.py gpurun_out/etr 60 > gpurun_out/ego_busy.txt
python tools/chains.py gpurun_out/etr > gpurun_out/ego_chains.txt
rm -rf gpurun_out/etr
cat gpurun_out/ego_chains.txt
