"""Per-trial cost of the D3 solve on an object-like problem: N edges on a small box seen at
10-20 m with exact flow (the bench's objects converge slowly: 100-200 LM iterations).  Run under
rocprofv3 --kernel-trace --stats; k_flow_lm's mean duration / iterations ~ time per iteration.
Usage: lm_trial_bench.py [N] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import multimot_track_amd as M  # noqa: E402
from synth_problems import K_KITTI, project, rot, se3  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 208
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rng = np.random.default_rng(5)
fx, fy, cx, cy = K_KITTI
Tl = se3(np.eye(3), np.zeros(3))
# object motion folded into the camera pose (D3 solves the object's apparent camera motion)
Tc = se3(rot([0.1, 1.0, 0.05], 0.01), np.array([0.05, 0.0, 0.6]))
box = np.stack([rng.uniform(-0.9, 0.9, n), rng.uniform(-0.75, 0.75, n),
                rng.uniform(-2.0, 2.0, n)], 1) + np.array([3.0, 0.5, 15.0])
uv, z = project(Tl, box, K_KITTI)
uv2, _ = project(Tc, box, K_KITTI)
obs = uv.astype(np.float32)
flow = (uv2 - uv).astype(np.float32)
ctx = M.Context(M.kitti03_config())
st = None
for _ in range(reps):
    st = ctx.flow_solve(obs, flow, z.astype(np.float32), Tl, Tl, 0.01, 0.5, 200, K_KITTI)
print("n=%d iterations=%d inliers=%d" % (n, st[2]["iterations"], st[2]["inliers"]), flush=True)
