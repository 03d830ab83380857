import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import multimot_track_amd as M  # noqa
from synth_problems import K_KITTI, flow_problem  # noqa
ctx = M.Context(M.kitti03_config(nfeatures=2000, max_batch=8))
obs, flow, depth, Tl, init, _ = flow_problem(1, 520, outlier_frac=0.1)
st = ctx.flow_solve(obs, flow, depth, Tl, init, 0.04, 0.3, 100, K_KITTI)
print(st[2], flush=True)
