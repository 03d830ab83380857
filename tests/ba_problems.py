"""Seeded synthetic LocalBundleAdjustment graphs (Optimizer.cc:3408-3541 shapes): keyframes along a
forward trajectory, map points in front of them, one edge per observation listed point by point in
keyframe order, stereo edges (uR = u - bf/z) mixed with monocular ones (uR = -1), ORB octaves with
their 1/sigma^2 information, pixel noise, perturbed initial estimates and gross outliers.  Inputs
only: expected outputs come from the CPU oracle (oracle/ba_ref.cpp) at test time."""
import numpy as np

from synth_problems import K_KITTI, rot, se3

BF = 387.5744
INV_SIGMA2 = (1.0 / (1.2 ** (2 * np.arange(8)))).astype(np.float32)


def ba_problem(seed, n_kf=6, n_fixed=2, n_pt=800, obs_per_pt=(1, 4), mono_frac=0.15,
               pix_noise=0.5, pose_noise=0.01, pt_noise=0.05, outlier_frac=0.03, kf0_local=True,
               K=K_KITTI, w=1242, h=375):
    """n_kf keyframe vertices (the first n_kf - n_fixed local, the rest fixed cameras; with
    kf0_local the first local one is keyframe 0, itself fixed) and n_pt points, each seen by a
    random run of consecutive keyframes.  Returns (problem dict, true poses, true points)."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    Tt = []
    for k in range(n_kf):
        R = rot([0, 1, 0], 0.01 * k + 0.002 * rng.normal())
        t = np.array([0.05 * rng.normal(), 0.02 * rng.normal(), -1.2 * k])
        Tt.append(se3(R, R @ t))
    Tt = np.stack(Tt)
    fixed = np.zeros(n_kf, np.uint8)
    fixed[n_kf - n_fixed:] = 1
    if kf0_local:
        fixed[0] = 1
    # points: seen from a reference keyframe at a random pixel and depth
    X = np.zeros((n_pt, 3))
    pts, kfs, obs, s = [], [], [], []
    for j in range(n_pt):
        k0 = rng.integers(0, n_kf)
        z = rng.uniform(4.0, 45.0)
        u0, v0 = rng.uniform(30, w - 30), rng.uniform(30, h - 30)
        pc = np.array([(u0 - cx) * z / fx, (v0 - cy) * z / fy, z])
        Twc = np.linalg.inv(Tt[k0].astype(np.float64))
        X[j] = Twc[:3, :3] @ pc + Twc[:3, 3]
        nobs = rng.integers(obs_per_pt[0], obs_per_pt[1] + 1)
        first = max(0, min(k0 - rng.integers(0, nobs), n_kf - nobs))
        for k in range(first, min(n_kf, first + nobs)):
            T = Tt[k].astype(np.float64)
            p = T[:3, :3] @ X[j] + T[:3, 3]
            if p[2] <= 0.5:
                continue
            u = p[0] / p[2] * fx + cx + rng.normal(scale=pix_noise)
            v = p[1] / p[2] * fy + cy + rng.normal(scale=pix_noise)
            if rng.uniform() < outlier_frac:
                u += rng.uniform(-25, 25)
                v += rng.uniform(-25, 25)
            ur = -1.0 if rng.uniform() < mono_frac else u - BF / p[2] + rng.normal(scale=pix_noise)
            octave = rng.integers(0, 8)
            pts.append(j)
            kfs.append(k)
            obs.append((u, v, ur))
            s.append(INV_SIGMA2[octave])
    T0 = Tt.copy()
    for k in range(n_kf):
        if not fixed[k]:
            dT = se3(rot(rng.normal(size=3), pose_noise * rng.normal()),
                     pose_noise * 5 * rng.normal(size=3))
            T0[k] = (dT.astype(np.float64) @ Tt[k]).astype(np.float32)
    X0 = X + rng.normal(scale=pt_noise, size=X.shape)
    P = dict(T=T0.astype(np.float32), fixed=fixed, X=X0.astype(np.float32),
             pt=np.array(pts, np.int32), kf=np.array(kfs, np.int32),
             obs=np.array(obs, np.float32).reshape(-1, 3), s=np.array(s, np.float32))
    return P, Tt, X.astype(np.float32)
