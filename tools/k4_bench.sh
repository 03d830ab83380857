set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --chunk 32 --seqs-per-gpu 4 --no-cpu > gpurun_out/bench_k4.json 2> gpurun_out/bench_k4.err
cat gpurun_out/bench_k4.json
