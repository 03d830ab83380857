# A/B in one box: LocalMapping stream priority (MMT_LM_PRIO 0 normal / 1 high / 2 low)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 0; do
  MMT_LM_PRIO=$v MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --chunk 64 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/r5p_$v.json 2> gpurun_out/r5p_$v.err
  echo "== prio $v $(python -c "import json;print(json.loads(open('gpurun_out/r5p_$v.json').read().strip().splitlines()[-1])['value'])")"
  grep "localmapping profile\]" gpurun_out/r5p_$v.err | head -2 | cut -c1-330
done
