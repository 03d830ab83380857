"""Matching problems (rows B3, C1-C3) built from the reference's kitti_sample frames.

Current/last frames are the oracle's ORB keypoints and descriptors of kitti_sample frames with
the fixture's disparity turned into depth (Tracking.cc:447-456); camera poses come from the CPU
oracle tracker.  MapPoints are back-projected last-frame keys (world position, the key's
descriptor with a few bits flipped, normal and distance invariance as MapPoint::
UpdateNormalAndDepth sets them, MapPoint.cc).  These are inputs only; expected outputs come from
the CPU oracle at test time."""
import numpy as np

from conftest import load_kitti_frame

K = (721.5377, 721.5377, 609.5593, 172.8540)
BF = 387.5744
W, H = 1242, 375
_CACHE = {}


def scale_factors(O):
    return O.orb_config()["scale"]


def depth_map(disp):
    dp = disp.astype(np.float32) / np.float32(256.0)
    with np.errstate(divide="ignore"):
        return (np.float32(BF) / dp).astype(np.float32)


def frame(O, i):
    key = ("frame", i)
    if key not in _CACHE:
        fr = load_kitti_frame(i)
        k, d = O.orb_extract(O.gray_from_bgr(fr["bgr"]), 2000)
        _CACHE[key] = (k, d, depth_map(fr["disp"]))
    return _CACHE[key]


def poses(O, n=3):
    """Tcw of kitti_sample frames 0..n-1 from the CPU oracle tracker."""
    key = ("poses", n)
    if key not in _CACHE:
        tr = O.Tracker(W, H, K, BF, 0, 2000)
        out = []
        for i in range(n):
            f = load_kitti_frame(i)
            out.append(tr.track(f["bgr"], f["disp"], f["flow"], f["sem"])["Tcw"].copy())
        _CACHE[key] = out
    return _CACHE[key]


def map_points(kps, desc, depth, Tcw, rng, flip_bits=8, max_depth=40.0):
    """Back-project keys with valid depth to world points (Frame::UnprojectStereo) and give them
    descriptors, normals and distance bounds.  Returns (Xw, mp_desc, valid, normal, dmin, dmax)."""
    n = len(kps)
    z = depth[kps["y"].astype(np.int32), kps["x"].astype(np.int32)]
    valid = (z > 0) & (z < max_depth)
    zz = np.where(valid, z, 1.0).astype(np.float32)
    xc = np.stack([(kps["x"] - K[2]) * zz / K[0], (kps["y"] - K[3]) * zz / K[1], zz], 1)
    Tinv = np.linalg.inv(Tcw.astype(np.float64))
    Xw = (xc.astype(np.float64) @ Tinv[:3, :3].T + Tinv[:3, 3]).astype(np.float32)
    md = desc.copy()
    for j in range(n):  # a few flipped bits: the MapPoint's distinctive descriptor differs
        bits = rng.integers(0, 256, rng.integers(0, flip_bits + 1))
        for b in bits:
            md[j, b >> 3] ^= np.uint8(1 << (b & 7))
    Ow = Tinv[:3, 3]
    PO = Xw.astype(np.float64) - Ow
    dist = np.linalg.norm(PO, axis=1)
    normal = (PO / np.maximum(dist, 1e-9)[:, None]).astype(np.float32)
    sc = np.float32(1.2) ** kps["octave"].astype(np.float32)
    dmax = (dist * sc).astype(np.float32)
    dmin = (dmax / np.float32(1.2 ** 7)).astype(np.float32)
    return Xw, md, valid, normal, dmin, dmax


def sbp_case(O, name, seed=0):
    """Inputs of SearchByProjection(Frame&, const Frame&, th, bMono) for a named case."""
    rng = np.random.default_rng(seed)
    T = poses(O)
    mono, check, th, dup = False, True, 15.0, 1
    if name == "forward":        # last 0 -> current 1 (camera moves forward: bForward)
        li, ci, Tl, Tc = 0, 1, T[0], T[1]
    elif name == "backward":     # last 1 -> current 0 (bBackward)
        li, ci, Tl, Tc = 1, 0, T[1], T[0]
    elif name == "still":        # same frame, small perturbation (neither)
        li, ci, Tl, Tc = 0, 0, T[0], T[0].copy()
        Tc[:3, 3] += np.array([0.02, -0.01, 0.1], np.float32)
        th = 7.0
    elif name == "mono_wide":    # bMono, the th = 2 * 15 retry window
        li, ci, Tl, Tc = 0, 1, T[0], T[1]
        mono, th = True, 30.0
    elif name == "no_orientation":
        li, ci, Tl, Tc = 1, 2, T[1], T[2]
        check = False
    elif name == "duplicates":   # 12 copies of each point: greedy conflicts and rescans
        li, ci, Tl, Tc = 0, 1, T[0], T[1]
        dup = 12
    elif name == "vo_points":    # 40 % temporal VO points (no observations): keys they bind stay open
        li, ci, Tl, Tc = 0, 1, T[0], T[1]
    elif name == "vo_duplicates":  # copies alternating VO / mapped: rebinding events, cleared keys
        li, ci, Tl, Tc = 0, 1, T[0], T[1]
        dup = 6
    elif name == "nan_points":   # points unprojected from depth +inf (NaN / inf coordinates)
        li, ci, Tl, Tc = 0, 1, T[0], T[1]
    else:
        raise KeyError(name)
    lk, ld, ldep = frame(O, li)
    ck, cd, cdep = frame(O, ci)
    Xw, md, valid, *_ = map_points(lk, ld, ldep, Tl, rng)
    active = valid & (rng.random(len(lk)) > 0.1)
    if dup > 1:
        sel = np.nonzero(active)[0][::7][:60]
        lk, Xw, md = np.repeat(lk[sel], dup), np.repeat(Xw[sel], dup, 0), np.repeat(md[sel], dup, 0)
        active = np.ones(len(lk), bool)
    obs = None
    if name == "vo_points":
        obs = (rng.random(len(lk)) > 0.4).astype(np.uint8)
    elif name == "vo_duplicates":
        obs = (np.arange(len(lk)) % 2).astype(np.uint8)
        # perturb some copies' angles so the rotation histogram rejects some events
        lk = lk.copy()
        lk["angle"][::5] = (lk["angle"][::5] + 97.0) % 360.0
    elif name == "nan_points":
        Xw = Xw.copy()
        Xw[::11] = np.nan
        Xw[5::13, 0] = np.inf
        Xw[7::17, 2] = np.inf
        active = active | (np.arange(len(lk)) % 11 == 0)
    return dict(kps=ck, desc=cd, depth=cdep, tcw=Tc, last_kps=lk, Xw=Xw, mp_desc=md,
                active=active.astype(np.uint8), tlw=Tl, th=th, mono=mono,
                check_orientation=check, obs=obs)


def local_case(O, name, seed=0):
    """Inputs of SearchLocalPoints / SearchByProjection(Frame&, vector<MapPoint*>, th)."""
    rng = np.random.default_rng(seed)
    T = poses(O)
    th, dup, taken_frac = 3.0, 1, 0.2
    if name == "rgbd":
        src, ci = [0, 2], 1
    elif name == "reloc_th5":
        src, ci = [0], 1
        th = 5.0
    elif name == "th1":
        src, ci = [2], 1
        th = 1.0
    elif name == "duplicates":
        src, ci = [0], 1
        dup, taken_frac = 10, 0.0
    else:
        raise KeyError(name)
    parts = []
    for si in src:
        k, d, dep = frame(O, si)
        Xw, md, valid, normal, dmin, dmax = map_points(k, d, dep, T[si], rng)
        sel = np.nonzero(valid)[0]
        parts.append((Xw[sel], md[sel], normal[sel], dmin[sel], dmax[sel]))
    Xw, md, normal, dmin, dmax = [np.concatenate(x) for x in zip(*parts)]
    if dup > 1:
        sel = np.arange(0, len(Xw), 9)[:80]
        Xw, md, normal, dmin, dmax = [np.repeat(a[sel], dup, 0) for a in (Xw, md, normal, dmin,
                                                                            dmax)]
    m = len(Xw)
    skip = (rng.random(m) < 0.1).astype(np.uint8) if dup == 1 else np.zeros(m, np.uint8)
    ck, cd, cdep = frame(O, ci)
    taken = (rng.random(len(ck)) < taken_frac).astype(np.uint8)
    return dict(kps=ck, desc=cd, depth=cdep, tcw=T[ci], Xw=Xw, normal=normal, min_dist=dmin,
                max_dist=dmax, pdesc=md, skip=skip, th=th, taken=taken)


SBP_CASES = ["forward", "backward", "still", "mono_wide", "no_orientation", "duplicates",
             "vo_points", "vo_duplicates", "nan_points"]
LOCAL_CASES = ["rgbd", "reloc_th5", "th1", "duplicates"]
