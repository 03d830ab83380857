"""Micro-benchmark of the flow-refined pose solve (mmt_pose_flow_solve probe) on synthetic
problems of the sizes the tracker sees; run under rocprofv3 --kernel-trace --stats to get the
per-launch kernel time.  MMT_LM_THREADS=<threads> forces the block size."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import multimot_track_amd as M  # noqa: E402
from synth_problems import K_KITTI, flow_problem  # noqa: E402

ctx = M.Context(M.kitti03_config())
for n, ego, reps in ((270, False, 20), (700, False, 20), (1600, True, 20)):
    obs, flow, depth, Tl, init, _ = flow_problem(11, n, outlier_frac=0.1)
    args = (0.04, 0.3, 100) if ego else (0.01, 0.5, 200)
    st = None
    t0 = time.perf_counter()
    for _ in range(reps):
        st = ctx.flow_solve(obs, flow, depth, Tl, init, *args, K_KITTI)
    dt = (time.perf_counter() - t0) / reps
    print("n=%d ego=%d iterations=%d inliers=%d host_ms_per_solve=%.3f" %
          (n, ego, st[2]["iterations"], st[2]["inliers"], dt * 1e3), flush=True)
