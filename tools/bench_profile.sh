# Round-end style measurement: bench line, rocprofv3 kernel stats of the same command, ORB traffic.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-cur}
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
cat gpurun_out/bench_$tag.json
rm -rf gpurun_out/benchk
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/benchk -o run -- python bench.py --no-cpu > gpurun_out/benchk.log 2>&1
python tools/rocprof_summary.py gpurun_out/benchk gpurun_out/bench_${tag}_kernel_stats.csv | grep "mmt::" | head -30
rm -rf gpurun_out/benchk
