"""The CPU oracle's LocalMapping steps against known answers:
LocalBundleAdjustment's solve (oracle/ba_ref.cpp; Optimizer.cc:3394-3665) on synthetic graphs, and
ORBmatcher::Fuse's per-point search (oracle/mapping_ref.cpp; ORBmatcher.cc:1200-1324) on a keyframe
built from the reference's kitti_sample frame.  The reference ships no fixtures for these
functions (parity unpinned); the known answers are geometric."""
import numpy as np
import pytest

from ba_problems import BF, ba_problem
from synth_problems import K_KITTI


def test_local_ba_noise_free_is_a_fixpoint(oracle_mod):
    """Exact observations at the true estimates: nothing moves beyond rounding and nothing is
    erased; the first round stops early (chi2 ~ 0)."""
    P, Tt, Xt = ba_problem(0, pix_noise=0.0, pose_noise=0.0, pt_noise=0.0, outlier_frac=0.0)
    P["T"], P["X"] = Tt.copy(), Xt.copy()
    T, X, er, st = oracle_mod.local_ba(P, K_KITTI, BF)
    assert er.sum() == 0
    assert np.abs(T - Tt).max() < 2e-5 and np.abs(X - Xt).max() < 2e-4


def test_local_ba_recovers_and_erases_outliers(oracle_mod):
    """Perturbed poses and points converge back towards the truth; fixed keyframes do not move
    (beyond the Converter round trip); gross outliers are among the erased edges."""
    P, Tt, Xt = ba_problem(1, n_pt=1200, pix_noise=0.3, outlier_frac=0.05)
    err0 = np.abs(P["T"] - Tt).max()
    T, X, er, st = oracle_mod.local_ba(P, K_KITTI, BF)
    fixed = P["fixed"].astype(bool)
    assert np.abs(T[fixed] - P["T"][fixed]).max() < 1e-6
    assert np.abs(T[~fixed] - Tt[~fixed]).max() < 0.2 * err0
    # edges whose observation was displaced by the generator's outlier step
    fx, fy, cx, cy = K_KITTI
    Tt64 = Tt.astype(np.float64)
    pc = np.einsum("eij,ej->ei", Tt64[P["kf"], :3, :3], Xt[P["pt"]].astype(np.float64)) + \
        Tt64[P["kf"], :3, 3]
    uv = np.stack([pc[:, 0] / pc[:, 2] * fx + cx, pc[:, 1] / pc[:, 2] * fy + cy], 1)
    # chi2 at the true estimates (the information 1/sigma^2 of the key's octave)
    chi_true = P["s"] * ((uv - P["obs"][:, :2]) ** 2).sum(1)
    # a point seen once can move onto its one observation; count the points seen at least twice
    multi = np.bincount(P["pt"], minlength=len(P["X"]))[P["pt"]] >= 2
    gross = (chi_true > 20.0) & multi
    assert gross.sum() > 10 and er[gross].mean() > 0.95
    assert er[chi_true < 2.0].mean() < 0.05
    assert st["iterations"][0] >= 1 and st["iterations"][1] >= 1


def test_local_ba_all_fixed_points_only(oracle_mod):
    """Only fixed keyframes: the solve still moves the points (the Schur system is empty)."""
    P, Tt, Xt = ba_problem(2, n_kf=3, n_fixed=3, n_pt=200, outlier_frac=0.0)
    T, X, er, st = oracle_mod.local_ba(P, K_KITTI, BF)
    assert np.abs(T - P["T"]).max() < 1e-6

    def cost(Xe):  # the edges' chi2 at the fixed poses, capped like a robust kernel
        fx, fy, cx, cy = K_KITTI
        Tk = T.astype(np.float64)[P["kf"]]
        pc = np.einsum("eij,ej->ei", Tk[:, :3, :3], Xe[P["pt"]].astype(np.float64)) + Tk[:, :3, 3]
        uv = np.stack([pc[:, 0] / pc[:, 2] * fx + cx, pc[:, 1] / pc[:, 2] * fy + cy], 1)
        return np.minimum(P["s"] * ((uv - P["obs"][:, :2]) ** 2).sum(1), 10.0).sum()

    assert cost(X) < 0.5 * cost(P["X"])


def _kitti_keyframe(kitti_frames, oracle_mod):
    f = kitti_frames[0]
    gray = oracle_mod.gray_from_bgr(f["bgr"])
    kps, desc = oracle_mod.orb_extract(gray, 2000)
    fx, fy, cx, cy = K_KITTI
    d = f["disp"].astype(np.float64)
    with np.errstate(divide="ignore"):
        depth = (BF / (d / 256.0)).astype(np.float32)
    return kps, desc, depth


def test_fuse_search_known_answers(kitti_frames, oracle_mod):
    """Points placed on keyframe keys (exact depth, the key's descriptor) find that key at
    distance 0 when its level is predicted (scale bounds built around the point's distance); a
    point behind the camera, one outside the image and one seen at more than 60 degrees find
    nothing."""
    kps, desc, depth = _kitti_keyframe(kitti_frames, oracle_mod)
    fx, fy, cx, cy = K_KITTI
    T = np.eye(4, dtype=np.float32)
    rng = np.random.default_rng(3)
    cand = [i for i in range(len(kps)) if np.isfinite(depth[int(kps[i]["y"]), int(kps[i]["x"])])]
    sel = rng.choice(cand, 40, replace=False)
    X, nrm, mind, maxd, pd = [], [], [], [], []
    for i in sel:
        u, v = float(kps[i]["x"]), float(kps[i]["y"])
        z = float(depth[int(v), int(u)])
        p = np.array([(u - cx) * z / fx, (v - cy) * z / fy, z])
        X.append(p)
        nrm.append(p / np.linalg.norm(p))
        dist = np.linalg.norm(p)
        lvl = int(kps[i]["octave"])
        mx = dist * 1.2 ** lvl  # mfMaxDistance as UpdateNormalAndDepth sets it for this level
        maxd.append(mx)
        mind.append(mx / 1.2 ** 7)
        pd.append(desc[i])
    X = np.array(X, np.float32)
    extra = [np.array([0, 0, -5.0]), np.array([1e3, 0, 10.0]), X[0].astype(np.float64)]
    extra_n = [np.array([0, 0, 1.0]), np.array([0, 0, 1.0]), -nrm[0]]
    X = np.vstack([X, np.array(extra, np.float32)])
    nrm = np.vstack([np.array(nrm), np.array(extra_n)]).astype(np.float32)
    mind = np.array(mind + [0.1, 0.1, mind[0]], np.float32)
    maxd = np.array(maxd + [1e4, 1e4, maxd[0]], np.float32)
    pd = np.vstack([np.array(pd), np.array(pd[:3])])
    idx, dist = oracle_mod.fuse_candidates(kps, desc, depth, T, X, nrm, mind, maxd, pd,
                                           K_KITTI, BF, 1242, 375)
    n = len(sel)
    ok = (dist[:n] == 0) & (idx[:n] == sel)
    assert ok.mean() > 0.9, (idx[:n], sel, dist[:n])
    assert (idx[n:] == -1).all() and (dist[n:] == 256).all()
