# Kernel trace of a short C3 bench (for the blit copies per frame): the trace CSV gzipped
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/etr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/etr -o run -- python bench.py --steps 3 --warmup 1 --chunk 64 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/r5za.log 2>&1
f="$(find /tmp/etr -name '*kernel_trace.csv' -print -quit)"
gzip -c "$f" > gpurun_out/r5za_trace.csv.gz
ls -la gpurun_out/r5za_trace.csv.gz
