"""Summarise MMT_LM_PROFILE lines (per-solve phase clocks) from a log: cycles per trial by phase,
split into small (N <= 500) and large solves.  Usage: lm_prof_parse.py <log>"""
import re
import sys
import collections

KEYS = ('schur_pass', 'schur_red', 'solve_ld', 'solve_ldlt', 'solve_exp', 'upd_pass', 'upd_red',
        'decide')
rows = []
for line in open(sys.argv[1]):
    if line.startswith('lmprof'):
        rows.append({k: int(v) for k, v in re.findall(r'(\w+)=(\d+)', line)})
for name, sel in (('small', lambda r: r['N'] <= 500), ('large', lambda r: r['N'] > 500)):
    rs = [r for r in rows if sel(r)]
    if not rs:
        continue
    tot = collections.Counter()
    for r in rs:
        for k in KEYS + ('trials', 'iters'):
            tot[k] += r[k]
    per = {k: round(tot[k] / tot['trials']) for k in KEYS}
    print("%s: %d solves, %.1f trials, %.1f iters, %d cycles/trial %s" % (
        name, len(rs), tot['trials'] / len(rs), tot['iters'] / len(rs),
        sum(tot[k] for k in KEYS) / tot['trials'], per))
