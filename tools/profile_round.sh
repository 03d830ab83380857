# The round's measurement record (argument: tag): the driver's bench command, then the same command
# under rocprofv3 --kernel-trace --stats (its kernel stats and its own bench line), into gpurun_out/
# for copying to profiles/.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
rm -rf gpurun_out/prof_$TAG
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py > gpurun_out/bench_${TAG}_under_rocprof.json 2> gpurun_out/bench_${TAG}_under_rocprof.err
python tools/rocprof_summary.py gpurun_out/prof_$TAG gpurun_out/kernel_stats_$TAG.csv | grep mmt | head -25
rm -rf gpurun_out/prof_$TAG
