"""Micro-benchmark of the PnP-RANSAC probe (mmt_pnp_ransac) at tracker-like sizes; run under
rocprofv3 --kernel-trace --stats for per-kernel times (MMT_PNP_PROFILE builds print phase cycles)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import multimot_track_amd as M  # noqa: E402
from synth_problems import K_KITTI, pnp_problem  # noqa: E402

ctx = M.Context(M.kitti03_config())
for n, out, reps in ((300, 0.0, 10), (700, 0.3, 10), (3000, 0.6, 10)):
    p3, p2, _ = pnp_problem(5, n, outlier_frac=out, pix_noise=0.05)
    t0 = time.perf_counter()
    for _ in range(reps):
        R, t, inl, info = ctx.pnp_ransac(p3, p2, K_KITTI)
    print("n=%d out=%.1f iterations=%d inliers=%d host_ms=%.3f" %
          (n, out, info["iterations"], len(inl), (time.perf_counter() - t0) / reps * 1e3), flush=True)
