# Where the vocabulary path's time goes: the default bench (vocabulary loaded) and the same run
# without it, both with MMT_MAP_PROFILE=1 (host stage times per frame and per keyframe on stderr).
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-vc}
common="--steps 8 --warmup 5 --no-cpu --single-frames 0 --c2-steps 0"
MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py $common > gpurun_out/${tag}_voc.json 2> gpurun_out/${tag}_voc.err
MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py $common --vocabulary '' > gpurun_out/${tag}_novoc.json 2> gpurun_out/${tag}_novoc.err
grep -h "profile\]" gpurun_out/${tag}_voc.err gpurun_out/${tag}_novoc.err
