"""D1 (Optimizer::PoseOptimization) kernel timing: repeated solves of synthetic problems of n edges
through mmt_pose_optimization; run under rocprofv3 --kernel-trace --stats for the kernel time.
Usage: python tools/d1_bench.py <n> [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import multimot_track_amd as M  # noqa: E402
from synth_problems import pose_opt_problem, K_KITTI  # noqa: E402

n = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
ctx = M.Context(M.kitti03_config(1242, 375, 2000))
Xw, obs, s2, init, _ = pose_opt_problem(7, n, outlier_frac=0.1, mono_frac=0.1)
for _ in range(reps):
    r = ctx.pose_optimization(Xw, obs, s2, init, K_KITTI, 387.5744)
print("n", n, "inliers", r[0])
ctx.close()
