"""Time the GPU local BA (mmt_local_bundle_adjustment) on synthetic graphs of the sizes the C3
sequence's LocalMapping builds (about 7 local keyframes, 3,000 points, 3,600 edges; bench.py's
local_mapping counters give the measured averages), and print µs per BA, per LM iteration and per
trial.  The host part of a call (graph layout, one upload, one download) is included, as in the
tracker.  Usage: python tools/ba_bench.py [--reps 20] [--pts 3000] [--kfs 9] [--fixed 2]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pts", type=int, default=3000)
    ap.add_argument("--kfs", type=int, default=9)
    ap.add_argument("--fixed", type=int, default=2)
    ap.add_argument("--obs", type=int, default=2, help="max observations per point")
    a = ap.parse_args()
    import multimot_track_amd as M
    from ba_problems import ba_problem
    ctx = M.Context(M.kitti03_config(nfeatures=2000))
    rows = []
    for seed in range(3):
        P, _, _ = ba_problem(seed, n_kf=a.kfs, n_fixed=a.fixed, n_pt=a.pts,
                             obs_per_pt=(1, a.obs))
        ctx.local_bundle_adjustment(P)  # warm: buffers sized, code loaded
        t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            _, _, _, st = ctx.local_bundle_adjustment(P)
            t.append(time.perf_counter() - t0)
        us = 1e6 * float(np.median(t))
        it, tr = sum(st["iterations"]), sum(st["trials"])
        rows.append(us)
        print("seed %d: %d kf (%d fixed), %d pts, %d edges: %.0f us per BA, %d iterations, %d "
              "trials, %.1f us per trial" % (seed, a.kfs, a.fixed, a.pts, len(P["pt"]), us, it, tr,
                                             us / max(tr, 1)), flush=True)
    ctx.close()
    print("median over seeds: %.0f us per BA" % float(np.median(rows)))


if __name__ == "__main__":
    main()
