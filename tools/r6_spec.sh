# Local map speculated during D1 (MMT_LOCALMAP_SPEC): the tracking / vocabulary / LocalMapping GPU
# tests first, then the 8-step bench under MMT_MAP_PROFILE=1 with and without, interleaved twice.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-spec}
timeout -k 10 900 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_vocab.py tests/test_gpu_localmap.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
common="--steps 8 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0"
for r in 1 2; do
  for sp in 1 0; do
    MMT_LOCALMAP_SPEC=$sp MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py $common > gpurun_out/${tag}_${sp}_$r.json 2> gpurun_out/${tag}_${sp}_$r.err
    python -c "import json,sys; d=json.load(open('gpurun_out/${tag}_${sp}_$r.json')); print('spec', $sp, 'round', $r, d['value'], d['valid'])"
    grep -h "map profile\] 16\|speculated" gpurun_out/${tag}_${sp}_$r.err
  done
done
