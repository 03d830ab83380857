set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf /tmp/tr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr -o run -- python bench.py --steps 6 --warmup 2 --no-cpu > gpurun_out/tr.log 2>&1
python tools/d3_gaps.py /tmp/tr
python tools/queue_busy.py /tmp/tr 100
