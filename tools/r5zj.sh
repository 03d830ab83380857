# Round-5 close-out (after the BA work): smoke(), the full GPU suite, the default bench line
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5zj_smoke.log 2>&1 || { tail -20 gpurun_out/r5zj_smoke.log; exit 1; }
tail -1 gpurun_out/r5zj_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r5zj_suite.log 2>&1 || { tail -40 gpurun_out/r5zj_suite.log; exit 1; }
tail -2 gpurun_out/r5zj_suite.log
timeout -k 10 600 python bench.py > gpurun_out/r5zj_bench.json 2> gpurun_out/r5zj_bench.err || { tail -20 gpurun_out/r5zj_bench.err; exit 1; }
cat gpurun_out/r5zj_bench.json
