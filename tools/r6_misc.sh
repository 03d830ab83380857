# Round-6 measurements: drift ablations (oracle, 2000 frames: depth_nearest, static, static_no_ba),
# bench --config C4 / C5 at N = 1, and several sequences per GPU (processes against contexts).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 560 python -u tools/drift_ablation.py --frames 2000 --configs depth_nearest,static,static_no_ba --out gpurun_out/drift2 > gpurun_out/drift2.log 2>&1
tail -3 gpurun_out/drift2.log
timeout -k 10 300 python bench.py --config C4 --steps 4 --warmup 1 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
for f in bench_c4 bench_c5; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['valid'], d['config']['workload'])"; done
