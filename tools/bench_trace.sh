set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/tr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/tr.log 2>&1
python tools/queue_busy.py gpurun_out/tr 100
