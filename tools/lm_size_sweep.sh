set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
export MMT_LIB_PATH=$PWD/multimot_track_amd/libmmt_lmprof.so
for n in 192 240 256 257 270 320 400 512; do
  timeout -k 10 60 python tools/lm_trial_bench.py $n 2 2>&1 | grep lmprof | tail -1 | python -c "
import sys,re
l=sys.stdin.read(); d=dict(re.findall(r'(\w+)=(\d+)',l)); d={k:int(v) for k,v in d.items()}
keys=('schur_pass','schur_red','solve_ld','solve_ldlt','solve_exp','upd_pass','upd_red','decide')
print('N=%d T=%d trials=%d iters=%d cycles/trial=%d' % (d['N'],d['T'],d['trials'],d['iters'],sum(d[k] for k in keys)/max(d['trials'],1)))"
done
