set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --chunk 32 --steps 40 --warmup 10 --no-cpu > gpurun_out/c32.json 2>/dev/null
timeout -k 10 300 python bench.py --chunk 64 --steps 20 --warmup 5 --no-cpu > gpurun_out/c64.json 2>/dev/null
for f in c32 c64; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f fps',d['value'],'orb_ms',d['roofline']['launch_ms'],'frac',d['roofline']['frac'],d['config']['frames_tracked'])"; done
