# Round-6 close-out on one box: the full GPU suite, smoke(), the default bench line, and the same
# bench command (shorter) under rocprofv3 --kernel-trace --stats, summarised on the box (kernel
# table + the batched ORB windows' spans, to set beside the line's HIP-event window).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-fin}
bash tools/r6_suite.sh $tag
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print('bench', d['value'], d['valid'], d['roofline']['frac'], d['roofline']['launch_ms'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${tag}_kt -o run -- python bench.py --steps 10 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/${tag}_kt_bench.json 2> gpurun_out/${tag}_kt_bench.err
python tools/rocpd_summary.py /tmp/${tag}_kt --mmt-only --orb-window 128 > gpurun_out/${tag}_kernel_stats.txt 2>&1
rm -rf /tmp/${tag}_kt
head -45 gpurun_out/${tag}_kernel_stats.txt
