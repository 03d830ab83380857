"""Debug: GPU flow solve vs oracle over a grid of problem parameters."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import multimot_track_amd as M  # noqa: E402
from oracle import oracle as O  # noqa: E402
from synth_problems import K_KITTI, flow_problem  # noqa: E402

ctx = M.Context(M.kitti03_config(nfeatures=2000, max_batch=8))
for seed, n, out, ego in [(1, 600, 0.1, True), (1, 600, 0.0, True), (1, 600, 0.1, False),
                          (1, 300, 0.1, True), (1, 500, 0.1, True), (1, 520, 0.1, True),
                          (1, 1100, 0.1, True), (2, 1500, 0.2, True), (2, 1500, 0.2, False)]:
    obs, flow, depth, Tl, init, _ = flow_problem(seed, n, outlier_frac=out)
    args = (0.04, 0.3, 100) if ego else (0.01, 0.5, 200)
    rc, pose_o, st_o = O.flow_solve(obs, flow, depth, Tl, init, *args, K_KITTI)
    status, pose_g, st_g = ctx.flow_solve(obs, flow, depth, Tl, init, *args, K_KITTI)
    print(seed, n, out, ego, "diff=%.2e" % np.abs(pose_g - pose_o).max(), "it", st_g["iterations"],
          st_o["iterations"], "inl", st_g["inliers"], st_o["inliers"], flush=True)
