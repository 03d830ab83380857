# D2 results written straight into pinned memory (MMT_D2_ZEROCOPY): tracking parity, then A/B
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_track.py -m gpu -x -q --timeout 240 --timeout-method thread -k "c3_long or lost_frame or synthetic or split or contexts" > gpurun_out/r5y_tests.log 2>&1 || { tail -30 gpurun_out/r5y_tests.log; exit 1; }
tail -1 gpurun_out/r5y_tests.log
for v in 1 0 1 0; do
  MMT_D2_ZEROCOPY=$v timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --single-frames 64 --c2-steps 2 > gpurun_out/r5y_$v.json 2> gpurun_out/r5y_$v.err
  echo "== zc=$v $(python -c "import json;d=json.loads(open('gpurun_out/r5y_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['c2']['value'], d['config']['one_frame_per_call']['ms_per_frame'])")"
done
