# A/B in one box: LocalMapping host blocks with the default library and with libmmt_prof.so
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in a b a b a b; do
  if [ $v = b ]; then L=multimot_track_amd/libmmt_prof.so; else L=multimot_track_amd/libmmt.so; fi
  MMT_LIB_PATH=$L MMT_MAP_PROFILE=1 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --chunk 64 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/r5o_$v.json 2> gpurun_out/r5o_$v.err
  echo "== $v $(python -c "import json;print(json.loads(open('gpurun_out/r5o_$v.json').read().strip().splitlines()[-1])['value'])")"
  grep "localmapping profile\]" gpurun_out/r5o_$v.err | tail -1 | cut -c1-400
done
