# rocprofv3 kernel stats of the driver's bench command (no CPU leg).  Usage: bench_prof.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-cur}
rm -rf gpurun_out/benchk
timeout -k 10 ${PROF_TIMEOUT:-1000} rocprofv3 --kernel-trace --stats -d gpurun_out/benchk -o run -- python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/benchk_$tag.json 2> gpurun_out/benchk.log
cat gpurun_out/benchk_$tag.json
python tools/rocprof_summary.py gpurun_out/benchk gpurun_out/bench_${tag}_kernel_stats.csv | grep "mmt::" | head -14
rm -rf gpurun_out/benchk
