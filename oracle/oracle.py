"""ctypes bindings for oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the
product (multimot_track_amd / libmmt.so) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        _LIB = ctypes.CDLL(path)
        _LIB.oracle_fast_atan2.restype = ctypes.c_float
        _LIB.oracle_fast_atan2.argtypes = [ctypes.c_float, ctypes.c_float]
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def orb_config(nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
    scale = np.zeros(nlevels, np.float32)
    sigma2 = np.zeros(nlevels, np.float32)
    npl = np.zeros(nlevels, np.int32)
    umax = np.zeros(16, np.int32)
    lib().oracle_orb_config(nfeatures, ctypes.c_float(scale_factor), nlevels, ini_th, min_th,
                            _p(scale), _p(sigma2), _p(npl), _p(umax))
    return dict(scale=scale, sigma2=sigma2, n_per_level=npl, umax=umax)


def level_sizes(w, h, nlevels=8, scale_factor=1.2):
    lw = np.zeros(nlevels, np.int32)
    lh = np.zeros(nlevels, np.int32)
    lib().oracle_level_sizes(1000, ctypes.c_float(scale_factor), nlevels, w, h, _p(lw), _p(lh))
    return lw, lh


def gray_from_bgr(bgr):
    bgr = np.ascontiguousarray(bgr, np.uint8)
    h, w = bgr.shape[:2]
    out = np.empty((h, w), np.uint8)
    lib().oracle_gray_from_bgr(_p(bgr), w, h, w * 3, _p(out))
    return out


def pyramid(gray, nlevels=8, scale_factor=1.2):
    gray = np.ascontiguousarray(gray, np.uint8)
    h, w = gray.shape
    lw, lh = level_sizes(w, h, nlevels, scale_factor)
    out = np.empty(int((lw.astype(np.int64) * lh).sum()), np.uint8)
    lib().oracle_pyramid(_p(gray), w, h, nlevels, ctypes.c_float(scale_factor), _p(out))
    levels, off = [], 0
    for a, b in zip(lw, lh):
        levels.append(out[off:off + a * b].reshape(b, a))
        off += a * b
    return levels


def blur7(img):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty_like(img)
    lib().oracle_blur7(_p(img), img.shape[1], img.shape[0], _p(out))
    return out


def fast_atan2(y, x):
    return lib().oracle_fast_atan2(float(y), float(x))


def level_candidates(level_img, ini_th=20, min_th=7):
    level_img = np.ascontiguousarray(level_img, np.uint8)
    cap = 1 << 20
    buf = np.empty((cap, 3), np.float32)
    n = lib().oracle_level_candidates(_p(level_img), level_img.shape[1], level_img.shape[0],
                                      ini_th, min_th, _p(buf), cap)
    assert n >= 0
    return buf[:n].copy()


def distribute(xyr, min_x, max_x, min_y, max_y, nfeat):
    xyr = np.ascontiguousarray(xyr, np.float32)
    cap = max(len(xyr), 1)
    out = np.empty((cap, 3), np.float32)
    n = lib().oracle_distribute(_p(xyr), len(xyr), min_x, max_x, min_y, max_y, nfeat, _p(out), cap)
    assert n >= 0
    return out[:n].copy()


def orb_extract(gray, nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
    gray = np.ascontiguousarray(gray, np.uint8)
    h, w = gray.shape
    cap = nfeatures * 4 + 1024
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_int(0)
    rc = lib().oracle_orb_extract(_p(gray), w, h, nfeatures, ctypes.c_float(scale_factor), nlevels,
                                  ini_th, min_th, _p(kps), _p(desc), cap, ctypes.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


# ------------------------------------------------------------------ tracker / solves
def rng_first_gaussian(seed):
    L = lib()
    L.oracle_rng_first_gaussian.restype = ctypes.c_float
    L.oracle_rng_first_gaussian.argtypes = [ctypes.c_ulonglong]
    return L.oracle_rng_first_gaussian(seed)


def flow_solve(obs, flow, depth, tcw_last, init, rp_thres, prior_info, max_iters, K):
    L = lib()
    L.oracle_flow_solve.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [
        ctypes.c_float, ctypes.c_double, ctypes.c_int] + [ctypes.c_float] * 4 + [ctypes.c_void_p] * 2
    obs = np.ascontiguousarray(obs, np.float32)
    flow = np.ascontiguousarray(flow, np.float32)
    depth = np.ascontiguousarray(depth, np.float32)
    tl = np.ascontiguousarray(tcw_last, np.float32).reshape(16)
    ini = np.ascontiguousarray(init, np.float32).reshape(16)
    pose = np.zeros(16, np.float32)
    st = np.zeros(6, np.int32)
    rc = L.oracle_flow_solve(len(depth), _p(obs), _p(flow), _p(depth), _p(tl), _p(ini), rp_thres,
                             prior_info, max_iters, K[0], K[1], K[2], K[3], _p(pose), _p(st))
    return rc, pose.reshape(4, 4), dict(iterations=int(st[0]), inliers=int(st[1]),
                                        rejections=int(st[3]), clean_rejections=int(st[4]),
                                        max_reject_run=int(st[5]))


def pose_optimization(Xw, obs, inv_sigma2, tcw, K, bf):
    """Optimizer::PoseOptimization (D1): returns (n_inliers, pose 4x4, outlier flags)."""
    L = lib()
    L.oracle_pose_optimization.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + \
        [ctypes.c_float] * 5 + [ctypes.c_void_p] * 2
    Xw = np.ascontiguousarray(Xw, np.float32)
    obs = np.ascontiguousarray(obs, np.float32)
    s2 = np.ascontiguousarray(inv_sigma2, np.float32)
    t = np.ascontiguousarray(tcw, np.float32).reshape(16)
    n = len(Xw)
    pose = np.zeros(16, np.float32)
    out = np.zeros(max(n, 1), np.uint8)
    rc = L.oracle_pose_optimization(n, _p(Xw), _p(obs), _p(s2), _p(t), K[0], K[1], K[2], K[3], bf,
                                    _p(pose), _p(out))
    return rc, pose.reshape(4, 4), out[:n].astype(bool)


def pnp_ransac(pts3, pts2, K, max_iters=500, reproj=0.3, conf=0.98):
    L = lib()
    L.oracle_pnp_ransac.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + \
        [ctypes.c_double] * 4 + [ctypes.c_int, ctypes.c_double, ctypes.c_double] + [ctypes.c_void_p] * 5
    pts3 = np.ascontiguousarray(pts3, np.float32)
    pts2 = np.ascontiguousarray(pts2, np.float32)
    n = len(pts3)
    R = np.zeros(9)
    t = np.zeros(3)
    inl = np.zeros(max(n, 1), np.int32)
    ninl = ctypes.c_int(0)
    its = np.zeros(2, np.int32)
    rc = L.oracle_pnp_ransac(_p(pts3), _p(pts2), n, K[0], K[1], K[2], K[3], max_iters, reproj,
                             conf, _p(R), _p(t), _p(inl), ctypes.byref(ninl), _p(its))
    return rc, R.reshape(3, 3), t, inl[:ninl.value].copy(), dict(iterations=int(its[0]),
                                                                 best_iter=int(its[1]))


def p4p_randi(n, iters, seed=1):
    """RandomInt(0, n-1-j) draws of a P4P RANSAC from glibc rand() seeded with `seed`."""
    out = np.zeros(max(iters, 1) * 4, np.int32)
    lib().oracle_p4p_randi(n, iters, ctypes.c_uint(seed), _p(out))
    return out[:iters * 4].reshape(iters, 4)


def glibc_rand(seed, count):
    out = np.zeros(count, np.int32)
    lib().oracle_glibc_rand(ctypes.c_uint(seed), count, _p(out))
    return out


def pnpsolver_iterate(pts3, pts2, sigma2, K, randi, n_iterations=5, state=None,
                      params=(0.99, 10, 300, 4, 0.5, 5.991)):
    """PnPsolver::SetRansacParameters(*params) + iterate(n_iterations) (oracle/pnp_ref.cpp).
    state: dict(iterations, best_inliers, best_Tcw (4x4), best_mask (n bool)), updated in place.
    Returns dict(found, no_more, n_inliers, Tcw, mask)."""
    L = lib()
    L.oracle_pnpsolver_iterate.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + \
        [ctypes.c_double] * 5 + [ctypes.c_int] * 3 + [ctypes.c_float] * 2 + \
        [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 6
    pts3 = np.ascontiguousarray(pts3, np.float32)
    pts2 = np.ascontiguousarray(pts2, np.float32)
    s2 = np.ascontiguousarray(sigma2, np.float32)
    n = len(pts3)
    if state is None:
        state = {}
    its = np.array([state.get("iterations", 0), state.get("best_inliers", 0)], np.int32)
    sT = np.ascontiguousarray(state.get("best_Tcw", np.zeros((4, 4))), np.float32).reshape(16)
    sm = np.ascontiguousarray(state.get("best_mask", np.zeros(n, bool)), np.uint8)
    ri = np.ascontiguousarray(randi, np.int32).reshape(-1)
    T = np.zeros(16, np.float32)
    m = np.zeros(max(n, 1), np.uint8)
    o3 = np.zeros(3, np.int32)
    # PnPsolver's fu, fv, uc, vc are doubles holding Frame's float fx, fy, cx, cy
    Kf = [float(np.float32(k)) for k in K]
    L.oracle_pnpsolver_iterate(_p(pts3), _p(pts2), _p(s2), n, Kf[0], Kf[1], Kf[2], Kf[3],
                               params[0], params[1], params[2], params[3], params[4], params[5],
                               _p(ri), n_iterations, _p(its), _p(sT), _p(sm), _p(T), _p(m),
                               _p(o3))
    state.update(iterations=int(its[0]), best_inliers=int(its[1]), best_Tcw=sT.reshape(4, 4),
                 best_mask=sm[:n].astype(bool))
    return dict(found=bool(o3[0]), no_more=bool(o3[1]), n_inliers=int(o3[2]),
                Tcw=T.reshape(4, 4), mask=m[:n].astype(bool))


def ransac_subsets(count, iters):
    out = np.zeros(iters * 5, np.int32)
    lib().oracle_ransac_subsets(count, iters, _p(out))
    return out.reshape(iters, 5)


_MAP_DUMP_FIELDS = (("kf_i", np.int64, 4), ("kf_T", np.float32, 16),
                    ("kf_mps_start", np.int32, 1), ("kf_mps", np.int32, 1),
                    ("pt_f", np.float32, 5), ("pt_i", np.int32, 5), ("obs_start", np.int32, 1),
                    ("obs_i", np.int32, 3), ("obs_f", np.float32, 4), ("conn", np.int32, 3),
                    ("ord", np.int32, 3), ("child", np.int32, 2))


class _MapDump(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k, _, _ in _MAP_DUMP_FIELDS]


def _map_dump_arrays(sizes):
    nk, npt, nob, nc, no, nch, nsl = (int(v) for v in sizes)
    rows = dict(kf_i=nk, kf_T=nk, kf_mps_start=nk + 1, kf_mps=nsl, pt_f=npt, pt_i=npt,
                obs_start=npt + 1, obs_i=nob, obs_f=nob, conn=nc, ord=no, child=nch)
    D = {k: np.zeros((max(rows[k], 1), w) if w > 1 else max(rows[k], 1), dt)
         for k, dt, w in _MAP_DUMP_FIELDS}
    st = _MapDump(**{k: D[k].ctypes.data_as(ctypes.c_void_p).value for k, _, _ in _MAP_DUMP_FIELDS})
    return {k: D[k][:rows[k]] for k in D}, D, st


BOW_STAT_KEYS = ("bow_frames", "trk", "trk_ok", "reloc", "reloc_ok", "reloc_cands", "pnp_found",
                 "sbp_rounds", "triangulated", "sft_matches", "kfdb")


class Vocabulary:
    """DBoW2 TemplatedVocabulary restated (oracle/bow_ref.cpp): loadFromTextFile, transform,
    score."""

    def __init__(self, path):
        L = lib()
        L.oracle_voc_load.restype = ctypes.c_void_p
        L.oracle_voc_load.argtypes = [ctypes.c_char_p]
        L.oracle_voc_free.argtypes = [ctypes.c_void_p]
        self._h = L.oracle_voc_load(path.encode())
        if not self._h:
            raise RuntimeError("oracle: cannot load vocabulary %s" % path)
        info = np.zeros(6, np.int32)
        L.oracle_voc_info(ctypes.c_void_p(self._h), _p(info))
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = (int(v) for v in info)

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.oracle_voc_free(self._h)
            self._h = None

    def transform(self, desc, levelsup=4):
        """-> dict(word, weight, node per feature; bow_word, bow_value; fv (ids, start, feat))."""
        desc = np.ascontiguousarray(desc, np.uint8)
        n = len(desc)
        m = max(n, 1)
        fw = np.zeros(m, np.uint32); fx = np.zeros(m, np.float64); fn = np.zeros(m, np.uint32)
        bw = np.zeros(m, np.uint32); bv = np.zeros(m, np.float64)
        fvn = np.zeros(m, np.uint32); fvs = np.zeros(m + 1, np.int32); fvf = np.zeros(m, np.int32)
        cnt = np.zeros(2, np.int32)
        lib().oracle_voc_transform(ctypes.c_void_p(self._h), _p(desc), n, levelsup, _p(fw), _p(fx),
                                   _p(fn), _p(bw), _p(bv), _p(fvn), _p(fvs), _p(fvf), _p(cnt))
        nb, nn = int(cnt[0]), int(cnt[1])
        return dict(word=fw[:n], weight=fx[:n], node=fn[:n], bow_word=bw[:nb], bow_value=bv[:nb],
                    fv=(fvn[:nn], fvs[:nn + 1], fvf[:fvs[nn]]))

    def score(self, a_word, a_value, b_word, b_value):
        L = lib()
        L.oracle_voc_score.restype = ctypes.c_double
        a_word = np.ascontiguousarray(a_word, np.uint32); b_word = np.ascontiguousarray(b_word, np.uint32)
        a_value = np.ascontiguousarray(a_value, np.float64); b_value = np.ascontiguousarray(b_value, np.float64)
        return float(L.oracle_voc_score(ctypes.c_void_p(self._h), _p(a_word), _p(a_value), len(a_word),
                                        _p(b_word), _p(b_value), len(b_word)))


class Tracker:
    """CPU restatement of System::TrackRGBD (oracle/track_ref.cpp)."""

    def __init__(self, w, h, K, bf, seed=0, nfeatures=2000):
        L = lib()
        L.oracle_tracker_create.restype = ctypes.c_void_p
        L.oracle_tracker_create.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_float] * 5 + \
            [ctypes.c_ulonglong, ctypes.c_int]
        L.oracle_tracker_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_tracker_track.argtypes = [ctypes.c_void_p] * 9 + [ctypes.c_int]
        self._h = L.oracle_tracker_create(w, h, K[0], K[1], K[2], K[3], bf, seed, nfeatures)

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.oracle_tracker_destroy(self._h)
            self._h = None

    def map_stats(self):
        """LocalMapping counters (oracle/mapping_ref.cpp)."""
        out = np.zeros(10, np.int64)
        lib().oracle_tracker_map_stats(ctypes.c_void_p(self._h), _p(out))
        keys = ("n_ba", "n_fused", "n_culled", "n_ba_erased", "ba_trials", "ba_edges", "ba_kfs",
                "ba_pts", "ba_max_opt_kfs", "n_reparent")
        return {k: int(v) for k, v in zip(keys, out)}

    def set_vocabulary(self, path):
        """System(voc, ...): run the reference's BoW steps (TrackReferenceKeyFrame,
        Relocalization, CreateNewMapPoints) with this DBoW2 text vocabulary."""
        L = lib()
        L.oracle_tracker_set_vocabulary.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        if L.oracle_tracker_set_vocabulary(self._h, path.encode()) != 0:
            raise RuntimeError("oracle: cannot load vocabulary %s" % path)

    def bow_stats(self):
        out = np.zeros(11, np.int64)
        lib().oracle_tracker_bow_stats(ctypes.c_void_p(self._h), _p(out))
        return dict(zip(BOW_STAT_KEYS, (int(v) for v in out)))

    def set_cull_ratio(self, r):
        """Test knob: KeyFrameCulling's redundancy ratio (0.9 in the reference)."""
        L = lib()
        L.oracle_tracker_set_cull_ratio.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.oracle_tracker_set_cull_ratio(self._h, float(r))

    def map_dump(self):
        """The map as flat arrays, in the layout of the product's mmt_map_dump (include/mmt.h)."""
        L = lib()
        sz = np.zeros(7, np.int32)
        h = ctypes.c_void_p(self._h)
        L.oracle_tracker_map_dump.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_tracker_map_dump(h, _p(sz), None)
        out, keep, st = _map_dump_arrays(sz)
        L.oracle_tracker_map_dump(h, _p(sz), ctypes.byref(st))
        del keep
        return out

    def capture_ba(self, which):
        """Record the problem of this tracker's which-th LocalBundleAdjustment (0-based)."""
        lib().oracle_tracker_capture_ba(ctypes.c_void_p(self._h), which)

    def captured_ba(self):
        """The captured LocalBundleAdjustment problem as a dict of arrays, or None."""
        L = lib()
        sz = np.zeros(3, np.int32)
        L.oracle_tracker_captured_ba(ctypes.c_void_p(self._h), _p(sz), None, None, None, None,
                                     None, None, None)
        nk, npt, ne = (int(v) for v in sz)
        if ne == 0 and nk == 0:
            return None
        P = dict(T=np.zeros((nk, 4, 4), np.float32), fixed=np.zeros(nk, np.uint8),
                 X=np.zeros((npt, 3), np.float32), pt=np.zeros(ne, np.int32),
                 kf=np.zeros(ne, np.int32), obs=np.zeros((ne, 3), np.float32),
                 s=np.zeros(ne, np.float32))
        L.oracle_tracker_captured_ba(ctypes.c_void_p(self._h), _p(sz), _p(P["T"]),
                                     _p(P["fixed"]), _p(P["X"]), _p(P["pt"]), _p(P["kf"]),
                                     _p(P["obs"]), _p(P["s"]))
        return P

    def capture_d3(self, frame, obj):
        """Record the D3 problem (PoseOptimizationFlow2 of one object) of object obj in this
        tracker's frame-th track() call (0-based)."""
        L = lib()
        L.oracle_tracker_capture_d3.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int]
        L.oracle_tracker_capture_d3(self._h, frame, obj)

    def captured_d3(self):
        """The captured D3 problem (obs, flow, depth, tcw_last, init as flow_solve takes them,
        with rp_thres 0.01, prior_info 0.5, max_iters 200), or None."""
        L = lib()
        n = np.zeros(1, np.int32)
        L.oracle_tracker_captured_d3(ctypes.c_void_p(self._h), _p(n), None, None, None, None, None)
        if n[0] < 0:
            return None
        m = int(n[0])
        P = dict(obs=np.zeros((m, 2), np.float32), flow=np.zeros((m, 2), np.float32),
                 depth=np.zeros(m, np.float32), tcw_last=np.zeros((4, 4), np.float32),
                 init=np.zeros((4, 4), np.float32))
        L.oracle_tracker_captured_d3(ctypes.c_void_p(self._h), _p(n), _p(P["obs"]), _p(P["flow"]),
                                     _p(P["depth"]), _p(P["tcw_last"]), _p(P["init"]))
        return P

    def track(self, bgr, disp, flow, mask):
        bgr = np.ascontiguousarray(bgr, np.uint8)
        disp = np.ascontiguousarray(disp, np.uint16)
        flow = np.ascontiguousarray(flow, np.float32)
        mask = np.ascontiguousarray(mask, np.int32)
        tcw = np.zeros(32, np.float32)
        info = np.zeros(13, np.int32)
        oi = np.zeros((16, 8), np.int32)
        of = np.zeros((16, 51), np.float32)
        lib().oracle_tracker_track(self._h, _p(bgr), _p(disp), _p(flow), _p(mask), _p(tcw),
                                   _p(info), _p(oi), _p(of), 16)
        objs = []
        for i in range(min(int(info[6]), 16)):
            objs.append(dict(label=int(oi[i, 0]), sem_label=int(oi[i, 1]), n_points=int(oi[i, 2]),
                             ransac_inliers=int(oi[i, 3]), mm_inliers=int(oi[i, 4]),
                             n_solve=int(oi[i, 5]), n_inliers=int(oi[i, 6]),
                             iterations=int(oi[i, 7]), init=of[i, :16].reshape(4, 4),
                             X=of[i, 16:32].reshape(4, 4), motion=of[i, 32:48].reshape(4, 4),
                             centre_pre=of[i, 48:51].copy()))
        return dict(initialized=bool(info[0]), Tcw=tcw[:16].reshape(4, 4), n_keys=int(info[1]),
                    n_static=int(info[2]), n_obj_samples=int(info[3]), ego_iterations=int(info[4]),
                    ego_inliers=int(info[5]), objects=objs, map_state=int(info[7]),
                    map_matches_mm=int(info[8]), map_inliers_local=int(info[9]),
                    n_keyframes=int(info[10]), n_mappoints=int(info[11]),
                    new_keyframe=int(info[12]), Tcw_map=tcw[16:].reshape(4, 4).copy())


def fuse_candidates(kps, desc, depth, tcw, Xw, normal, min_dist, max_dist, pdesc, K, bf,
                    w, h, nfeatures=2000, th=3.0):
    """ORBmatcher::Fuse's per-point search against one keyframe (oracle/mapping_ref.cpp):
    (best key index, best distance) per point, -1 / 256 for none."""
    c = orb_config(nfeatures)
    scale = np.ascontiguousarray(c["scale"], np.float32)
    inv_s2 = np.ascontiguousarray(np.float32(1.0) / c["sigma2"], np.float32)  # 1.0f / sigma2
    kps = np.ascontiguousarray(kps)
    desc = np.ascontiguousarray(desc, np.uint8)
    depth = np.ascontiguousarray(depth, np.float32)
    tcw = np.ascontiguousarray(tcw, np.float32)
    arrs = [np.ascontiguousarray(a, np.float32) for a in (Xw, normal, min_dist, max_dist)]
    pd = np.ascontiguousarray(pdesc, np.uint8)
    m = len(arrs[2])
    idx = np.zeros(max(m, 1), np.int32)
    dist = np.zeros(max(m, 1), np.int32)
    cam = np.array([K[0], K[1], K[2], K[3], bf], np.float32)
    lib().oracle_fuse_candidates(w, h, _p(cam), len(scale), _p(scale), _p(inv_s2), len(kps),
                                 _p(kps), _p(desc), _p(depth), _p(tcw), m, _p(arrs[0]),
                                 _p(arrs[1]), _p(arrs[2]), _p(arrs[3]), _p(pd),
                                 ctypes.c_float(th), _p(idx), _p(dist))
    return idx[:m], dist[:m]


def local_ba(P, K, bf):
    """Optimizer::LocalBundleAdjustment's solve (oracle/ba_ref.cpp) on a problem dict (the keys of
    Tracker.captured_ba).  Returns (T (n_kf, 4, 4), X (n_pt, 3), erase (n_edge,), stats dict)."""
    nk, npt, ne = len(P["fixed"]), len(P["X"]), len(P["pt"])
    T = np.ascontiguousarray(P["T"], np.float32)
    X = np.ascontiguousarray(P["X"], np.float32)
    To = np.zeros((nk, 4, 4), np.float32)
    Xo = np.zeros((npt, 3), np.float32)
    er = np.zeros(max(ne, 1), np.uint8)
    st = np.zeros(5, np.int32)
    cam = np.array([K[0], K[1], K[2], K[3], bf], np.float32)
    lib().oracle_local_ba(nk, npt, ne, _p(T), _p(np.ascontiguousarray(P["fixed"], np.uint8)),
                          _p(X), _p(np.ascontiguousarray(P["pt"], np.int32)),
                          _p(np.ascontiguousarray(P["kf"], np.int32)),
                          _p(np.ascontiguousarray(P["obs"], np.float32)),
                          _p(np.ascontiguousarray(P["s"], np.float32)), _p(cam), _p(To), _p(Xo),
                          _p(er), _p(st))
    stats = dict(iterations=(int(st[0]), int(st[1])), trials=(int(st[2]), int(st[3])),
                 n_erase=int(st[4]))
    return To, Xo, er[:ne], stats


# ---------------------------------------------------------------- B3 / C1-C3 (match_ref.cpp)
def _cam(K, bf):
    return np.array([K[0], K[1], K[2], K[3], bf], np.float32)


def frame_stereo_grid(kps, depth, K, bf):
    """Frame::ComputeStereoFromRGBD + AssignFeaturesToGrid: (uR, depth, cell_start, cell_idx)."""
    L = lib()
    L.oracle_frame_stereo_grid.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    depth = np.ascontiguousarray(depth, np.float32)
    H, W = depth.shape
    n = len(kps)
    uR = np.zeros(max(n, 1), np.float32)
    dep = np.zeros(max(n, 1), np.float32)
    cs = np.zeros(64 * 48 + 1, np.int32)
    ci = np.zeros(max(n, 1), np.int32)
    cam = _cam(K, bf)
    tot = L.oracle_frame_stereo_grid(n, _p(kps), _p(depth), W, H, _p(cam), _p(uR), _p(dep),
                                     _p(cs), _p(ci))
    return uR[:n], dep[:n], cs, ci[:tot]


def search_by_projection_frame(kps, desc, depth, tcw, last_kps, Xw, mp_desc, active, tlw, th,
                               K, bf, scale, mono=False, check_orientation=True, obs=None):
    L = lib()
    vp = ctypes.c_void_p
    L.oracle_search_by_projection_frame.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int,
                                                    ctypes.c_int, vp, vp, ctypes.c_int, vp,
                                                    ctypes.c_int, vp, vp, vp, vp, vp,
                                                    ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                                    vp, vp]
    ob = None if obs is None else np.ascontiguousarray(obs, np.uint8)
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    depth = np.ascontiguousarray(depth, np.float32)
    H, W = depth.shape
    lk = np.ascontiguousarray(last_kps, KP_DTYPE)
    X = np.ascontiguousarray(Xw, np.float32)
    md = np.ascontiguousarray(mp_desc, np.uint8)
    act = np.ascontiguousarray(active, np.uint8)
    sc = np.ascontiguousarray(scale, np.float32)
    t = np.ascontiguousarray(tcw, np.float32).reshape(16)
    tl = np.ascontiguousarray(tlw, np.float32).reshape(16)
    cam = _cam(K, bf)
    match = np.zeros(max(len(kps), 1), np.int32)
    nm = L.oracle_search_by_projection_frame(len(kps), _p(kps), _p(desc), _p(depth), W, H,
                                             _p(cam), _p(sc), len(sc), _p(t), len(lk), _p(lk),
                                             _p(X), _p(md), _p(act), _p(tl), th, int(mono),
                                             int(check_orientation), _p(match),
                                             None if ob is None else _p(ob))
    return nm, match[:len(kps)]


def search_by_bow(kf_fv, kf_kps, kf_desc, kf_mp_ok, f_fv, f_kps, f_desc, nnratio=0.7,
                  check_orientation=True):
    """C4 SearchByBoW(KeyFrame*, Frame&): kf_fv / f_fv = (node ids ascending, starts, features)."""
    L = lib()
    vp = ctypes.c_void_p
    L.oracle_search_by_bow.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_int, vp, vp,
                                       vp, ctypes.c_int, vp, vp, ctypes.c_float, ctypes.c_int, vp]

    def fv(v):
        node, start, feat = v
        return (np.ascontiguousarray(node, np.uint32), np.ascontiguousarray(start, np.int32),
                np.ascontiguousarray(feat, np.int32))
    kn, ks, kf = fv(kf_fv)
    fn, fs, ff = fv(f_fv)
    kk = np.ascontiguousarray(kf_kps, KP_DTYPE)
    kd = np.ascontiguousarray(kf_desc, np.uint8)
    ok = np.ascontiguousarray(kf_mp_ok, np.uint8)
    fk = np.ascontiguousarray(f_kps, KP_DTYPE)
    fd = np.ascontiguousarray(f_desc, np.uint8)
    match = np.zeros(max(len(fk), 1), np.int32)
    nm = L.oracle_search_by_bow(len(kn), _p(kn), _p(ks), _p(kf), _p(kk), _p(kd), _p(ok), len(fn),
                                _p(fn), _p(fs), _p(ff), len(fk), _p(fk), _p(fd), nnratio,
                                int(check_orientation), _p(match))
    return nm, match[:len(fk)]


def search_local_points(kps, desc, depth, tcw, Xw, normal, min_dist, max_dist, pdesc, skip, th,
                        K, bf, scale, taken=None):
    L = lib()
    vp = ctypes.c_void_p
    L.oracle_search_local_points.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int,
                                             ctypes.c_int, vp, vp, ctypes.c_int, vp,
                                             ctypes.c_int, vp, vp, vp, vp, vp, vp,
                                             ctypes.c_float, vp, vp, vp]
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    depth = np.ascontiguousarray(depth, np.float32)
    H, W = depth.shape
    arrs = [np.ascontiguousarray(a, np.float32) for a in (Xw, normal, min_dist, max_dist)]
    pd = np.ascontiguousarray(pdesc, np.uint8)
    sk = np.ascontiguousarray(skip, np.uint8)
    m = len(sk)
    tk = np.zeros(max(len(kps), 1), np.uint8) if taken is None else \
        np.ascontiguousarray(taken, np.uint8)
    sc = np.ascontiguousarray(scale, np.float32)
    t = np.ascontiguousarray(tcw, np.float32).reshape(16)
    cam = _cam(K, bf)
    match = np.zeros(max(len(kps), 1), np.int32)
    frus = np.zeros((max(m, 1), 6), np.float32)
    nm = L.oracle_search_local_points(len(kps), _p(kps), _p(desc), _p(depth), W, H, _p(cam),
                                      _p(sc), len(sc), _p(t), m, *[_p(a) for a in arrs], _p(pd),
                                      _p(sk), th, _p(tk), _p(match), _p(frus))
    return nm, match[:len(kps)], frus[:m]
