# Sequences per GPU: K contexts in one process (--seqs-per-gpu) against R processes
# (--ranks-per-gpu), 1-GPU box.  Usage: bash tools/r6_rpg.sh <tag> [K...]
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-rpg}
shift || true
common="--steps 6 --warmup 1 --no-cpu --single-frames 0 --c2-steps 0 --rank-parity-frames 64"
for k in ${@:-4 8}; do
  timeout -k 10 400 python bench.py --ranks-per-gpu $k $common > gpurun_out/${tag}_r$k.json 2> gpurun_out/${tag}_r$k.err
  timeout -k 10 400 python bench.py --seqs-per-gpu $k $common > gpurun_out/${tag}_k$k.json 2> gpurun_out/${tag}_k$k.err
done
for f in gpurun_out/${tag}_*.json; do
  python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['config']['sequences_per_gpu'], d['config'].get('ranks_per_gpu'), d['frames_tracked'], d['frames_timed'], [ (r['first_divergent_frame'], r['frames']) for r in (d.get('rank_parity') or [])])"
done
