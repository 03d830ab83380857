# Several sequences per GPU with the final round-5 build (K = 4, 8), rank/sequence parity records
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 4 8; do
  timeout -k 10 500 python bench.py --seqs-per-gpu $k --steps 4 --warmup 1 --no-cpu --single-frames 0 --c2-steps 0 > gpurun_out/r5zk_k$k.json 2> gpurun_out/r5zk_k$k.err || { tail -20 gpurun_out/r5zk_k$k.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5zk_k$k.json').read().strip().splitlines()[-1]);print('K=$k', d['value'], d['valid'], d['frames_tracked'], d['frames_timed'], [ (r['sequence'], r.get('first_divergent_frame')) for r in (d.get('rank_parity') or [])])"
done
