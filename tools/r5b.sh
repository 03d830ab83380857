# round 5: new tests (flush ordering, BA past 128 rows, map graph), then several sequences per GPU
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_track.py tests/test_gpu_localmap.py -m gpu -x -v --timeout 240 --timeout-method thread -k "partial_flush or local_ba_matches or map_graph or deferred" > gpurun_out/r5b_tests.log 2>&1 || { tail -40 gpurun_out/r5b_tests.log; exit 1; }
tail -3 gpurun_out/r5b_tests.log
for K in 4 8; do
timeout -k 10 500 python bench.py --seqs-per-gpu $K --steps 6 --warmup 2 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/r5b_k$K.json 2> gpurun_out/r5b_k$K.err || { tail -20 gpurun_out/r5b_k$K.err; exit 1; }
cat gpurun_out/r5b_k$K.json
done
