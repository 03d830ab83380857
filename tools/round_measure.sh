# Round measurement: parity tests, ORB traffic (PMC passes) for the bench batch, the bench line
# (driver flags), and the rocprofv3 kernel stats of the same bench command.  Usage: round_measure.sh <tag>
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-cur}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/orb_traffic.sh ${TRAFFIC_B:-128} | tail -4
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
cat gpurun_out/bench_$tag.json
[ "${PROF:-1}" = 0 ] && exit 0
rm -rf gpurun_out/benchk
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/benchk -o run -- python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/benchk_$tag.json 2> gpurun_out/benchk.log
python tools/rocprof_summary.py gpurun_out/benchk gpurun_out/bench_${tag}_kernel_stats.csv | grep "mmt::" | head -12
rm -rf gpurun_out/benchk
