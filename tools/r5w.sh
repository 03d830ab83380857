# D1 with 256-thread workgroups (libmmt_prof.so, MMT_PO_THREADS=256) against 512: D1 tests, then
# the bench (no CPU leg) alternately
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MMT_LIB_PATH=multimot_track_amd/libmmt_prof.so timeout -k 10 300 python -u -m pytest tests/test_gpu_track.py -m gpu -x -q --timeout 240 --timeout-method thread -k "pose_optimization or c3_long" > gpurun_out/r5w_tests.log 2>&1 || { tail -30 gpurun_out/r5w_tests.log; exit 1; }
tail -1 gpurun_out/r5w_tests.log
for v in a b a b; do
  if [ $v = b ]; then L=multimot_track_amd/libmmt_prof.so; else L=multimot_track_amd/libmmt.so; fi
  MMT_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --single-frames 0 --c2-steps 2 > gpurun_out/r5w_$v.json 2> gpurun_out/r5w_$v.err
  echo "== $v $(python -c "import json;d=json.loads(open('gpurun_out/r5w_$v.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['c2']['value'])")"
done
