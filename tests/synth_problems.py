"""Seeded synthetic inputs for single-solve parity tests (flow-refined pose LM, PnP-RANSAC).

These are inputs only; expected outputs come from the CPU oracle (oracle/) at test time."""
import numpy as np

K_KITTI = (721.5377, 721.5377, 609.5593, 172.8540)


def rot(axis, ang):
    axis = np.asarray(axis, np.float64)
    axis = axis / np.linalg.norm(axis)
    k = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * k + (1 - np.cos(ang)) * k @ k


def se3(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T.astype(np.float32)


def project(T, Pw, K):
    fx, fy, cx, cy = K
    pc = (T[:3, :3].astype(np.float64) @ Pw.T).T + T[:3, 3]
    return np.stack([pc[:, 0] / pc[:, 2] * fx + cx, pc[:, 1] / pc[:, 2] * fy + cy], 1), pc[:, 2]


def flow_problem(seed, n, outlier_frac=0.1, pix_noise=0.3, motion=0.05, K=K_KITTI,
                 w=1242, h=375):
    """A last-frame pose, a true current pose, n world points seen in both; returns
    (obs, flow, depth, Tcw_last, init, T_true).  Flow carries pixel noise and outliers."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    Tl = se3(rot(rng.normal(size=3), 0.05 * rng.normal()), rng.normal(size=3))
    dT = se3(rot(rng.normal(size=3), motion * 0.1 * rng.normal()),
             np.array([0.02, 0.01, 1.0]) * motion * 20 * rng.normal(size=3))
    Tc = (dT.astype(np.float64) @ Tl).astype(np.float32)
    u = rng.uniform(20, w - 20, n)
    v = rng.uniform(20, h - 20, n)
    z = rng.uniform(3.0, 40.0, n)
    pc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    Twl = np.linalg.inv(Tl.astype(np.float64))
    Pw = (Twl[:3, :3] @ pc.T).T + Twl[:3, 3]
    uv2, _ = project(Tc, Pw, K)
    flow = uv2 - np.stack([u, v], 1) + rng.normal(scale=pix_noise, size=(n, 2))
    nout = int(outlier_frac * n)
    if nout:
        flow[:nout] += rng.uniform(-30, 30, size=(nout, 2))
    obs = np.stack([u, v], 1).astype(np.float32)
    # initial estimate: last pose (constant position) as in the tracker's second frame
    return (obs, flow.astype(np.float32), z.astype(np.float32), Tl, Tl.copy(), Tc)


def pnp_problem(seed, n, outlier_frac=0.3, pix_noise=0.1, K=K_KITTI):
    """n 3-D points in the last camera frame and their pixels in the current frame."""
    rng = np.random.default_rng(seed)
    T = se3(rot(rng.normal(size=3), 0.1 * rng.normal()), rng.normal(size=3) * [0.3, 0.1, 1.0])
    p = np.stack([rng.uniform(-8, 8, n), rng.uniform(-2, 2, n), rng.uniform(6, 30, n)], 1)
    uv, z = project(T, p, K)
    uv += rng.normal(scale=pix_noise, size=uv.shape)
    nout = int(outlier_frac * n)
    if nout:
        uv[-nout:] += rng.uniform(-40, 40, size=(nout, 2))
    return p.astype(np.float32), uv.astype(np.float32), T


def pose_opt_problem(seed, n, outlier_frac=0.1, pix_noise=0.8, mono_frac=0.2, K=K_KITTI,
                     bf=387.5744):
    """Frame observations of n MapPoints for Optimizer::PoseOptimization: world points, undistorted
    keypoints with octave-scaled noise, right coordinates (uR = u - bf/z, or -1 for mono), the
    per-octave information 1/sigma^2 (ORB scale 1.2) and a perturbed initial pose."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    T = se3(rot(rng.normal(size=3), 0.05 * rng.normal()), rng.normal(size=3))
    u = rng.uniform(20, 1222, n)
    v = rng.uniform(20, 355, n)
    z = rng.uniform(4.0, 40.0, n)
    pc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    Tinv = np.linalg.inv(T.astype(np.float64))
    Xw = ((Tinv[:3, :3] @ pc.T).T + Tinv[:3, 3]).astype(np.float32)
    octave = rng.integers(0, 8, n)
    scale = 1.2 ** octave
    inv_sigma2 = (1.0 / (scale * scale)).astype(np.float32)
    uo = u + rng.normal(scale=pix_noise, size=n) * scale
    vo = v + rng.normal(scale=pix_noise, size=n) * scale
    ur = uo - bf / z
    mono = rng.uniform(size=n) < mono_frac
    ur[mono] = -1.0
    nout = int(outlier_frac * n)
    if nout:
        uo[:nout] += rng.uniform(-40, 40, nout)
        vo[:nout] += rng.uniform(-40, 40, nout)
    obs = np.stack([uo, vo, ur], 1).astype(np.float32)
    dT = se3(rot(rng.normal(size=3), 0.02 * rng.normal()), rng.normal(size=3) * 0.1)
    init = (dT.astype(np.float64) @ T.astype(np.float64)).astype(np.float32)
    return Xw, obs, inv_sigma2, init, T


def p4p_problem(seed, n, outlier_frac=0.3, pix_noise=0.5, K=K_KITTI):
    """Relocalization-style PnPsolver input (row D6): n MapPoint world positions, their keypoint
    pixels in the current frame (octave-scaled noise; an outlier fraction moved by up to 60 px)
    and mvLevelSigma2[octave] (ORB scale 1.2); returns (pts3, pts2, sigma2, Tcw_true)."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    T = se3(rot(rng.normal(size=3), 0.2 * rng.normal()), rng.normal(size=3) * [1.0, 0.2, 2.0])
    u = rng.uniform(20, 1222, n)
    v = rng.uniform(20, 355, n)
    z = rng.uniform(4.0, 40.0, n)
    pc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    Tinv = np.linalg.inv(T.astype(np.float64))
    Xw = ((Tinv[:3, :3] @ pc.T).T + Tinv[:3, 3]).astype(np.float32)
    octave = rng.integers(0, 8, n)
    scale = 1.2 ** octave
    sigma2 = (scale * scale).astype(np.float32)
    uv = np.stack([u, v], 1) + rng.normal(scale=pix_noise, size=(n, 2)) * scale[:, None]
    nout = int(outlier_frac * n)
    if nout:
        idx = rng.choice(n, nout, replace=False)
        uv[idx] += rng.uniform(-60, 60, size=(nout, 2))
    return Xw, uv.astype(np.float32), sigma2, T
