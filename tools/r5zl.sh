# Local BA kernel stats of the final round-5 build (rocprofv3 --kernel-trace over tools/ba_bench.py)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf /tmp/r5zl_trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5zl_trace -o run -- python tools/ba_bench.py --reps 8 > gpurun_out/r5zl_trace.log 2>&1 || { tail -20 gpurun_out/r5zl_trace.log; exit 1; }
cp "$(find /tmp/r5zl_trace -name '*kernel_stats.csv' -print -quit)" gpurun_out/r5zl_kernel_stats.csv
grep -E "ba2|Name" gpurun_out/r5zl_kernel_stats.csv | cut -d, -f1-5
