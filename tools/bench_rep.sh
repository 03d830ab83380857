# Parity tests, then the bench line N times (run-to-run spread).  Usage: bench_rep.sh [N]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for r in $(seq 1 ${1:-2}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_rep$r.json 2> gpurun_out/bench_rep$r.err
  python -c "import json;d=json.load(open('gpurun_out/bench_rep$r.json'));print('fps',d['value'],'orb_ms',d['roofline']['launch_ms'],'frac',d['roofline']['frac'])"
done
