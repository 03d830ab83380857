"""Per-frame cost of each object's D3 solve from an MMT_LM_PROFILE log (lmprof lines with blk and
stats): the launch time is set by the slowest object of the frame.  Prints the sum over frames of
the per-frame maximum against the largest per-object sum (what independent per-object chains
would need), in trial-cycles.  Usage: d3_objects.py <log>"""
import re
import sys

launches = []
cur, key = [], None
for line in open(sys.argv[1]):
    if not line.startswith("lmprof"):
        continue
    d = dict(re.findall(r"(\w+)=(\S+)", line))
    if int(d["iters"]) < 30 and int(d["N"]) > 150 and d.get("blk") is not None and \
            int(d["trials"]) < 40:
        continue  # the ego solve (split slices) and short solves
    cyc = sum(int(d[k]) for k in ("schur_pass", "schur_red", "solve_ld", "solve_ldlt",
                                  "solve_exp", "upd_pass", "upd_red", "decide"))
    base = int(d["stats"], 16) - 12 * int(d["blk"])
    if base != key and cur:
        launches.append(cur)
        cur = []
    key = base
    cur.append((int(d["blk"]), int(d["N"]), int(d["trials"]), cyc))
if cur:
    launches.append(cur)
per_obj = {}
s_max = 0
for L in launches:
    s_max += max(c for _, _, _, c in L)
    for b, n, t, c in L:
        per_obj[b] = per_obj.get(b, 0) + c
print("launches", len(launches), "objects per launch", sorted(set(len(L) for L in launches)))
print("sum of per-launch max: %.1f Mcycles" % (s_max / 1e6))
for b in sorted(per_obj):
    print("object slot %d: sum %.1f Mcycles" % (b, per_obj[b] / 1e6))
worst = sum(1 for L in launches for b, n, t, c in L if c == max(x[3] for x in L))
