# Host wait mode, interleaved in one process (MMT_SCHED: 0 the runtime's heuristic, 1 spin, 2 yield)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_interleave.py --rounds 5 'MMT_SCHED=0' 'MMT_SCHED=1' 'MMT_SCHED=2' > gpurun_out/r5zc.txt 2>&1
tail -12 gpurun_out/r5zc.txt
