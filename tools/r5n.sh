# LocalMapping host blocks (MMT_MAP_PROFILE) of a short C3 bench
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py --steps 6 --warmup 1 --chunk 64 --no-cpu --single-frames 0 > gpurun_out/r5n_prof.json 2> gpurun_out/r5n_prof.err
grep "profile\]" gpurun_out/r5n_prof.err | head -7
