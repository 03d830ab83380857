# Where the previous frame's object path runs: during the C2 chain (with the local map speculated
# there too) or during the C3 chain (MMT_OVERLAP_C3=1); 8-step bench, interleaved twice.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ovl}
common="--steps 8 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0"
for r in ${ROUNDS:-1 2}; do
  for o in 0 1; do
    MMT_OVERLAP_C3=$o MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py $common > gpurun_out/${tag}_${o}_$r.json 2> gpurun_out/${tag}_${o}_$r.err
    python -c "import json,sys; d=json.load(open('gpurun_out/${tag}_${o}_$r.json')); print('overlap_c3', $o, 'round', $r, d['value'], d['valid'])"
    grep -h "map profile\] 16\|tracker profile\] 16" gpurun_out/${tag}_${o}_$r.err
  done
done
