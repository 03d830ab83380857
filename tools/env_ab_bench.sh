# GPU tests, then the driver's bench line by default and under each environment setting named.
# Usage: env_ab_bench.sh <tag> [VAR=value ...]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
tag=$1; shift
i=0
for v in default "$@"; do
  out=gpurun_out/bench_${tag}_$i
  if [ "$v" = default ]; then
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > $out.json 2> $out.err
  else
    env "$v" timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > $out.json 2> $out.err
  fi
  echo "$v: $(python -c "import json;d=json.load(open('$out.json'));print(d['value'], d['roofline']['launch_ms'])")"
  i=$((i+1))
done
