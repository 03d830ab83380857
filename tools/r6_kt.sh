# The default bench command (shorter) under rocprofv3 --kernel-trace --stats, summarised on the box
# (kernel table + the batched ORB windows' spans) with a heartbeat while the summary runs.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-kt}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${tag}_kt -o run -- python bench.py --steps 6 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
python tools/rocpd_summary.py /tmp/${tag}_kt --mmt-only --orb-window 128 > gpurun_out/${tag}_kernel_stats.txt 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do echo "summary running $(date +%T)"; sleep 30; done
wait $pid
rm -rf /tmp/${tag}_kt
head -50 gpurun_out/${tag}_kernel_stats.txt
