# Host wait mode A/B: the runtime default, ROC_ACTIVE_WAIT_TIMEOUT (spin before the interrupt
# wait) and hipDeviceScheduleSpin / Yield (MMT_SCHED), one box, C3 + C2 + one frame per call
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu --single-frames 128 --c2-steps 2 > gpurun_out/r5zb_$tag.json 2> gpurun_out/r5zb_$tag.err
  echo "== $tag $(python -c "import json;d=json.loads(open('gpurun_out/r5zb_$tag.json').read().strip().splitlines()[-1]);print(d['value'], d['config']['c2']['value'], d['config']['one_frame_per_call']['ms_per_frame'])")"
}
run base A=0
run aw1000 ROC_ACTIVE_WAIT_TIMEOUT=1000
run spin MMT_SCHED=1
run base2 A=0
run aw1000b ROC_ACTIVE_WAIT_TIMEOUT=1000
run spin2 MMT_SCHED=1
run yield MMT_SCHED=2
