# Close-out without the profiler: the full GPU suite, smoke() and the default bench line.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-close}
bash tools/r6_suite.sh $tag
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print('bench', d['value'], d['valid'], d['roofline']['frac'], d['roofline']['launch_ms'], d['parity']['first_divergent_frame'], d['parity']['int_mismatch_frames'])"
