# The bench line (C3 value, C2 value) under each environment setting named, no tests.
# Usage: env_ab_quick.sh <tag> [VAR=value ...]   (VAR=value,VAR2=value2 sets several)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
i=0
for v in default "$@"; do
  out=gpurun_out/abq_${tag}_$i
  if [ "$v" = default ]; then
    timeout -k 10 300 python bench.py --no-cpu > $out.json 2> $out.err
  else
    env ${v//,/ } timeout -k 10 300 python bench.py --no-cpu > $out.json 2> $out.err
  fi
  echo "$v: $(python -c "import json;d=json.load(open('$out.json'));print(d['value'], d['config']['c2']['value'])")"
  i=$((i+1))
done
