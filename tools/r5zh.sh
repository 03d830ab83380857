# Object path: statistics download and PnP records + subset upload as one copy each; tracking parity
# (object paths included), then the in-box A/B against the previous library (libmmt_prev.so)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_pnpsolver.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5zh_tests.log 2>&1 || { tail -30 gpurun_out/r5zh_tests.log; exit 1; }
tail -1 gpurun_out/r5zh_tests.log
for v in new prev new prev new prev; do
  if [ $v = prev ]; then export MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_prev.so; else unset MMT_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --single-frames 128 --c2-steps 2 > gpurun_out/r5zh_$v.json 2> gpurun_out/r5zh_$v.err
  echo "== $v $(python -c "import json;d=json.loads(open('gpurun_out/r5zh_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['c2']['value'], d['config']['one_frame_per_call']['ms_per_frame'], d['valid'])")"
done
