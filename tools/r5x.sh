# D1 dual light pass (MMT_PO_DUAL): D1 / tracking parity tests, then the bench with and without
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_localmap.py -m gpu -x -q --timeout 240 --timeout-method thread -k "pose_optimization or c3_long or lost_frame or map_graph or synthetic" > gpurun_out/r5x_tests.log 2>&1 || { tail -30 gpurun_out/r5x_tests.log; exit 1; }
tail -1 gpurun_out/r5x_tests.log
for v in 1 0 1 0; do
  MMT_PO_DUAL=$v timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --single-frames 0 --c2-steps 2 > gpurun_out/r5x_$v.json 2> gpurun_out/r5x_$v.err
  echo "== dual=$v $(python -c "import json;d=json.loads(open('gpurun_out/r5x_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['c2']['value'])")"
done
