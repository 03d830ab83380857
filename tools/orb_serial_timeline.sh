set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf /tmp/rz
MMT_ORB_SCHED=2 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/rz -o run -- python tools/orb_microbench.py 64 5 > gpurun_out/rz.log 2>&1
python tools/timeline.py /tmp/rz 0.9 | tail -20
