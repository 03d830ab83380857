# bench at 64- and 128-frame chunks over the same frames (640-3199), no CPU baseline
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --chunk 128 --steps 20 --warmup 5 --no-cpu > gpurun_out/c128.json 2>/dev/null
timeout -k 10 400 python bench.py --chunk 64 --steps 40 --warmup 10 --no-cpu > gpurun_out/c64b.json 2>/dev/null
for f in c128 c64b; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f fps',d['value'],'orb_ms',d['roofline']['launch_ms'],'frac',d['roofline']['frac'],d['config']['frames_tracked'],d['config']['scene_render_s'])"; done
