# bench --config C4 / C5 at N = 1 on the current build (vocabulary loaded).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config C4 --steps 4 --warmup 1 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
for f in bench_c4 bench_c5; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['valid'], d['config']['workload'])"; done
