"""multimot_track_amd -- MI355X-native per-frame front end of cule/multimot_track.

The product is libmmt.so (HIP kernels for gfx950 + C++ host code behind the C-ABI of
include/mmt.h).  This Python module is thin ctypes plumbing over that C-ABI for tests, bench.py
and scripting; it has no compute path of its own and raises if libmmt.so is missing.

The ORBextractor class mirrors the reference interface ORB_SLAM2::ORBextractor
(include/ORBextractor.h:44-111 of the reference): constructor arguments, operator() ->
(keypoints, descriptors), GetLevels/GetScaleFactor/GetScaleFactors/... accessors.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MMT_LIB_PATH") or os.path.join(_HERE, "libmmt.so")  # override: tools/ (profiling builds)
_LIB = None

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class MmtConfig(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("k1", ctypes.c_float), ("k2", ctypes.c_float),
                ("p1", ctypes.c_float), ("p2", ctypes.c_float), ("k3", ctypes.c_float),
                ("bf", ctypes.c_float), ("th_depth", ctypes.c_float), ("rgb", ctypes.c_int),
                ("orb_nfeatures", ctypes.c_int), ("orb_scale_factor", ctypes.c_float),
                ("orb_nlevels", ctypes.c_int), ("orb_ini_th_fast", ctypes.c_int),
                ("orb_min_th_fast", ctypes.c_int), ("noise_seed", ctypes.c_uint32),
                ("device_id", ctypes.c_int), ("max_batch", ctypes.c_int),
                ("fps", ctypes.c_float)]


class MmtMotion(ctypes.Structure):
    _fields_ = [("label", ctypes.c_int32), ("sem_label", ctypes.c_int32),
                ("n_points", ctypes.c_int32), ("n_inliers", ctypes.c_int32),
                ("n_ransac_inliers", ctypes.c_int32), ("n_mm_inliers", ctypes.c_int32),
                ("n_solve", ctypes.c_int32), ("iterations", ctypes.c_int32),
                ("world_motion", ctypes.c_float * 16), ("cam_pose", ctypes.c_float * 16),
                ("init_pose", ctypes.c_float * 16), ("centre_pre", ctypes.c_float * 3)]


class MmtFrameResult(ctypes.Structure):
    _fields_ = [("Tcw", ctypes.c_float * 16), ("initialized", ctypes.c_int32),
                ("n_keypoints", ctypes.c_int32), ("n_obj_samples", ctypes.c_int32),
                ("ego_iterations", ctypes.c_int32), ("ego_inliers", ctypes.c_int32),
                ("n_objects", ctypes.c_int32), ("map_state", ctypes.c_int32),
                ("map_matches_mm", ctypes.c_int32), ("map_inliers_local", ctypes.c_int32),
                ("n_keyframes", ctypes.c_int32), ("n_mappoints", ctypes.c_int32),
                ("new_keyframe", ctypes.c_int32), ("Tcw_map", ctypes.c_float * 16),
                ("frame_index", ctypes.c_int32), ("objects_frame", ctypes.c_int32)]


class MmtFlowProblem(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("obs", ctypes.c_void_p), ("flow", ctypes.c_void_p),
                ("depth", ctypes.c_void_p), ("Tcw_last", ctypes.c_float * 16),
                ("init", ctypes.c_float * 16), ("rp_thres", ctypes.c_float),
                ("prior_info", ctypes.c_double), ("max_iters", ctypes.c_int),
                ("use_noise", ctypes.c_int), ("g0", ctypes.c_float), ("fx", ctypes.c_float),
                ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float)]


class MmtPoseOptProblem(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("Xw", ctypes.c_void_p), ("obs", ctypes.c_void_p),
                ("inv_sigma2", ctypes.c_void_p), ("Tcw", ctypes.c_float * 16),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("bf", ctypes.c_float)]


class MmtMatchFrame(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("kps", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("depth", ctypes.c_void_p), ("Tcw", ctypes.c_float * 16)]


class MmtLastFrame(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("kps", ctypes.c_void_p), ("Xw", ctypes.c_void_p),
                ("mp_desc", ctypes.c_void_p), ("active", ctypes.c_void_p),
                ("Tcw", ctypes.c_float * 16), ("obs", ctypes.c_void_p)]


class MmtLocalPoints(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int), ("Xw", ctypes.c_void_p), ("normal", ctypes.c_void_p),
                ("min_dist", ctypes.c_void_p), ("max_dist", ctypes.c_void_p),
                ("desc", ctypes.c_void_p), ("skip", ctypes.c_void_p)]


class MmtPnPsolverProblem(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("pts3", ctypes.c_void_p), ("pts2", ctypes.c_void_p),
                ("sigma2", ctypes.c_void_p), ("fx", ctypes.c_float), ("fy", ctypes.c_float),
                ("cx", ctypes.c_float), ("cy", ctypes.c_float), ("probability", ctypes.c_double),
                ("min_inliers", ctypes.c_int), ("max_iterations", ctypes.c_int),
                ("min_set", ctypes.c_int), ("epsilon", ctypes.c_float), ("th2", ctypes.c_float)]


class MmtPnPsolverState(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int), ("best_inliers", ctypes.c_int),
                ("best_Tcw", ctypes.c_float * 16), ("best_mask", ctypes.c_void_p)]


class MmtBAProblem(ctypes.Structure):
    _fields_ = [("n_kf", ctypes.c_int), ("n_pt", ctypes.c_int), ("n_edge", ctypes.c_int),
                ("Tcw", ctypes.c_void_p), ("fixed", ctypes.c_void_p), ("Xw", ctypes.c_void_p),
                ("e_pt", ctypes.c_void_p), ("e_kf", ctypes.c_void_p), ("e_obs", ctypes.c_void_p),
                ("e_inv_sigma2", ctypes.c_void_p)]


class MmtMapCounters(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in (
        "n_ba", "n_fused", "n_culled", "n_ba_erased", "ba_trials", "ba_edges", "ba_kfs",
        "ba_pts", "ba_max_opt", "fuse_launches", "fuse_queries", "fuse_relaunches")] + \
        [(k, ctypes.c_double) for k in ("lm_us", "ba_us", "fuse_us")] + \
        [("d2_split_fallbacks", ctypes.c_int64), ("n_reparent", ctypes.c_int64)]


class MmtBowCounters(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in ("bow_frames", "trk", "trk_ok", "reloc", "reloc_ok",
                                               "reloc_cands", "pnp_found", "sbp_rounds",
                                               "triangulated", "sft_matches", "kfdb")]


MAP_DUMP_FIELDS = (("kf_i", np.int64, 4), ("kf_T", np.float32, 16), ("kf_mps_start", np.int32, 1),
                   ("kf_mps", np.int32, 1), ("pt_f", np.float32, 5), ("pt_i", np.int32, 5),
                   ("obs_start", np.int32, 1), ("obs_i", np.int32, 3), ("obs_f", np.float32, 4),
                   ("conn", np.int32, 3), ("ord", np.int32, 3), ("child", np.int32, 2))


class MmtMapDumpArrays(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k, _, _ in MAP_DUMP_FIELDS]


def map_dump_arrays(sizes):
    """numpy arrays for mmt_map_dump's sizes[7] (keyframes, points, observations, connections,
    ordered covisibles, children, keyframe slots) and the struct pointing at them."""
    nk, npt, nob, nc, no, nch, nsl = (int(v) for v in sizes)
    rows = dict(kf_i=nk, kf_T=nk, kf_mps_start=nk + 1, kf_mps=nsl, pt_f=npt, pt_i=npt,
                obs_start=npt + 1, obs_i=nob, obs_f=nob, conn=nc, ord=no, child=nch)
    D = {k: np.zeros((max(rows[k], 1), w) if w > 1 else max(rows[k], 1), dt)
         for k, dt, w in MAP_DUMP_FIELDS}
    st = MmtMapDumpArrays(**{k: D[k].ctypes.data_as(ctypes.c_void_p).value
                             for k, _, _ in MAP_DUMP_FIELDS})
    return {k: D[k][:rows[k]] for k in D}, D, st


class MmtProfile(ctypes.Structure):
    _fields_ = [("orb_ms", ctypes.c_double), ("orb_launches", ctypes.c_int64),
                ("orb_frames", ctypes.c_int64)]


MAX_OBJECTS = 15  # objects reported per frame (kMaxObj in csrc/mmt_tracker.h: labels 1..15)


def _mat(a):
    return np.array(a[:], np.float32).reshape(4, 4)


def _frame_dict(r, objs):
    """Same keys as oracle.Tracker.track so tests compare like for like."""
    out = []
    for o in objs[:r.n_objects]:
        out.append(dict(label=o.label, sem_label=o.sem_label, n_points=o.n_points,
                        ransac_inliers=o.n_ransac_inliers, mm_inliers=o.n_mm_inliers,
                        n_solve=o.n_solve, n_inliers=o.n_inliers, iterations=o.iterations,
                        init=_mat(o.init_pose), X=_mat(o.cam_pose), motion=_mat(o.world_motion),
                        centre_pre=np.array(o.centre_pre[:], np.float32)))
    return dict(initialized=bool(r.initialized), Tcw=_mat(r.Tcw), n_keys=r.n_keypoints,
                n_obj_samples=r.n_obj_samples, ego_iterations=r.ego_iterations,
                ego_inliers=r.ego_inliers, objects=out, map_state=r.map_state,
                map_matches_mm=r.map_matches_mm, map_inliers_local=r.map_inliers_local,
                n_keyframes=r.n_keyframes, n_mappoints=r.n_mappoints,
                new_keyframe=r.new_keyframe, Tcw_map=_mat(r.Tcw_map),
                frame_index=r.frame_index, objects_frame=r.objects_frame)


class MmtError(RuntimeError):
    pass


class MmtFeatureVector(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int), ("node_id", ctypes.c_void_p),
                ("node_start", ctypes.c_void_p), ("feat", ctypes.c_void_p)]


class MmtBowKeyFrame(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("kps", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("mp_valid", ctypes.c_void_p), ("fv", MmtFeatureVector)]


def _feature_vector(v, keep):
    """(node ids ascending, starts (n_nodes + 1), features) -> MmtFeatureVector."""
    node, start, feat = (np.ascontiguousarray(v[0], np.uint32), np.ascontiguousarray(v[1], np.int32),
                         np.ascontiguousarray(v[2], np.int32))
    keep += [node, start, feat]
    fv = MmtFeatureVector()
    fv.n_nodes = len(node)
    fv.node_id, fv.node_start, fv.feat = node.ctypes.data, start.ctypes.data, feat.ctypes.data
    return fv


def lib():
    """Load libmmt.so; fail loudly (no fallback) when the HIP extension is not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise MmtError("libmmt.so not built: run `python -c 'import __graft_entry__ as g; "
                           "g.build()'` (there is no CPU fallback)")
        try:
            # torch's bundled HIP runtime carries the same SONAME (libamdhip64.so.7): loading it
            # first makes libmmt bind to it, so one runtime serves both and torch device
            # pointers / streams are valid in libmmt.  Loaded the other way round, two HIP
            # runtimes end up in the process and torch no longer sees the GPU.
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(os.environ.get("MMT_LIB_PATH", LIB_PATH))  # override: A/B builds
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.mmt_version.restype = i32
        L.mmt_last_error.restype = ctypes.c_char_p
        L.mmt_last_error.argtypes = [vp]
        L.mmt_create.restype = vp
        L.mmt_create.argtypes = [ctypes.POINTER(MmtConfig)]
        L.mmt_destroy.argtypes = [vp]
        L.mmt_orb_levels.argtypes = [vp, vp, vp, vp, vp, vp]
        L.mmt_orb_capacity.argtypes = [vp]
        L.mmt_orb_extract.argtypes = [vp, vp, i32, i32, i32, vp, vp, i32, vp]
        L.mmt_orb_extract_batch.argtypes = [vp, vp, i32, i32, vp, vp, i32, vp]
        L.mmt_orb_extract_device.argtypes = [vp, vp, i32, sz, vp, vp, i32, vp, vp]
        L.mmt_orb_device_status.argtypes = [vp, vp]
        L.mmt_debug_orb_raise.argtypes = [vp, i32]
        L.mmt_debug_fetch.restype = ctypes.c_long
        L.mmt_debug_fetch.argtypes = [vp, i32, i32, vp, sz]
        L.mmt_reset.argtypes = [vp]
        L.mmt_track_rgbd.argtypes = [vp, vp, vp, vp, vp, ctypes.c_double, vp, vp, i32]
        L.mmt_track_rgbd_chunk_device.argtypes = [vp, i32, vp, sz, vp, sz, vp, sz, vp, sz, vp, vp,
                                                  i32, vp]
        L.mmt_pose_flow_solve.argtypes = [vp, ctypes.POINTER(MmtFlowProblem), vp, vp]
        L.mmt_pose_optimization.argtypes = [vp, ctypes.POINTER(MmtPoseOptProblem), vp, vp, vp]
        L.mmt_pnp_ransac.argtypes = [vp, vp, vp, i32] + [ctypes.c_float] * 4 + \
            [i32, ctypes.c_double, ctypes.c_double] + [vp] * 5
        L.mmt_pnpsolver_iterate.argtypes = [vp, ctypes.POINTER(MmtPnPsolverProblem), vp, i32,
                                            i32, ctypes.POINTER(MmtPnPsolverState), vp, vp, vp,
                                            vp, vp]
        L.mmt_frame_grid.argtypes = [vp, ctypes.POINTER(MmtMatchFrame), vp, vp, vp, vp]
        L.mmt_search_by_projection_frame.argtypes = [vp, ctypes.POINTER(MmtMatchFrame),
                                                     ctypes.POINTER(MmtLastFrame),
                                                     ctypes.c_float, i32, i32, vp, vp]
        L.mmt_search_local_points.argtypes = [vp, ctypes.POINTER(MmtMatchFrame),
                                              ctypes.POINTER(MmtLocalPoints), ctypes.c_float,
                                              vp, vp, vp, vp]
        L.mmt_search_by_bow.argtypes = [vp, ctypes.POINTER(MmtBowKeyFrame), i32, vp, vp,
                                        ctypes.POINTER(MmtFeatureVector), ctypes.c_float, i32,
                                        vp, vp]
        L.mmt_profile_enable.argtypes = [vp, i32]
        L.mmt_profile_read.argtypes = [vp, ctypes.POINTER(MmtProfile), i32]
        L.mmt_fuse_candidates.argtypes = [vp, ctypes.POINTER(MmtMatchFrame),
                                          ctypes.POINTER(MmtLocalPoints), ctypes.c_float, vp, vp]
        L.mmt_local_bundle_adjustment.argtypes = [vp, ctypes.POINTER(MmtBAProblem), vp, vp, vp,
                                                  vp]
        L.mmt_map_counters_read.argtypes = [vp, ctypes.POINTER(MmtMapCounters)]
        L.mmt_map_dump.argtypes = [vp, vp, ctypes.POINTER(MmtMapDumpArrays)]
        L.mmt_set_keyframe_culling_ratio.argtypes = [vp, ctypes.c_double]
        L.mmt_load_vocabulary.argtypes = [vp, ctypes.c_char_p]
        L.mmt_bow_transform.argtypes = [vp, vp, i32, i32, vp, vp, vp]
        L.mmt_bow_counters_read.argtypes = [vp, ctypes.POINTER(MmtBowCounters)]
        L.mmt_set_deferred_objects.argtypes = [vp, i32]
        L.mmt_flush_objects.argtypes = [vp, vp, vp, i32, i32, vp]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def kitti03_config(width=1242, height=375, nfeatures=2000, max_batch=1, device_id=0,
                   noise_seed=0):
    """Settings of the reference's kitti_sample/kitti03.yaml (nFeatures overridable)."""
    c = MmtConfig()
    c.width, c.height = width, height
    c.fx, c.fy, c.cx, c.cy = 721.5377, 721.5377, 609.5593, 172.8540
    c.bf, c.th_depth, c.rgb, c.fps = 387.5744, 65.2, 1, 10.0
    c.orb_nfeatures, c.orb_scale_factor, c.orb_nlevels = nfeatures, 1.2, 8
    c.orb_ini_th_fast, c.orb_min_th_fast = 20, 7
    c.noise_seed, c.device_id, c.max_batch = noise_seed, device_id, max_batch
    return c


class Context:
    """Owns one mmt_ctx (one HIP device + stream)."""

    def __init__(self, cfg):
        self.cfg = cfg
        self._h = lib().mmt_create(ctypes.byref(cfg))
        if not self._h:
            raise MmtError("mmt_create failed: %s" % lib().mmt_last_error(None).decode())
        self.nlevels = cfg.orb_nlevels

    def close(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.mmt_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc < 0:
            raise MmtError("libmmt error %d: %s" % (rc, lib().mmt_last_error(self._h).decode()))
        return rc

    @property
    def handle(self):
        return self._h

    def capacity(self):
        return self._check(lib().mmt_orb_capacity(self._h))

    def levels(self):
        n = self.nlevels
        scale = np.zeros(n, np.float32)
        sigma2 = np.zeros(n, np.float32)
        npl = np.zeros(n, np.int32)
        lw = np.zeros(n, np.int32)
        lh = np.zeros(n, np.int32)
        self._check(lib().mmt_orb_levels(self._h, _p(scale), _p(sigma2), _p(npl), _p(lw), _p(lh)))
        return dict(scale=scale, sigma2=sigma2, n_per_level=npl, level_w=lw, level_h=lh)

    def orb_extract(self, gray):
        gray = np.ascontiguousarray(gray, np.uint8)
        h, w = gray.shape
        cap = self.capacity()
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int(0)
        self._check(lib().mmt_orb_extract(self._h, _p(gray), w, h, w, _p(kps), _p(desc), cap,
                                          ctypes.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def orb_extract_batch(self, grays):
        grays = [np.ascontiguousarray(g, np.uint8) for g in grays]
        h, w = grays[0].shape
        cap = self.capacity()
        nf = len(grays)
        ptrs = (ctypes.c_void_p * nf)(*[g.ctypes.data for g in grays])
        kps = np.zeros((nf, cap), KP_DTYPE)
        desc = np.zeros((nf, cap, 32), np.uint8)
        ns = np.zeros(nf, np.int32)
        self._check(lib().mmt_orb_extract_batch(self._h, ptrs, nf, w, _p(kps), _p(desc), cap,
                                                _p(ns)))
        return [(kps[i, :ns[i]].copy(), desc[i, :ns[i]].copy()) for i in range(nf)]

    # -- tracking (System::TrackRGBD) ---------------------------------------------------------
    def reset(self):
        self._check(lib().mmt_reset(self._h))

    def track(self, bgr, disp, flow, mask, timestamp=0.0):
        """One RGB-D frame: BGR u8 HxWx3, disparity*256 u16 HxW, flow f32 HxWx2, labels i32 HxW."""
        bgr = np.ascontiguousarray(bgr, np.uint8)
        disp = np.ascontiguousarray(disp, np.uint16)
        flow = np.ascontiguousarray(flow, np.float32)
        mask = np.ascontiguousarray(mask, np.int32)
        h, w = disp.shape
        assert (w, h) == (self.cfg.width, self.cfg.height), "frame size differs from the context"
        assert bgr.shape == (h, w, 3) and flow.shape == (h, w, 2) and mask.shape == (h, w)
        r = MmtFrameResult()
        objs = (MmtMotion * MAX_OBJECTS)()
        self._check(lib().mmt_track_rgbd(self._h, _p(bgr), _p(disp), _p(flow), _p(mask),
                                         float(timestamp), ctypes.byref(r), objs, MAX_OBJECTS))
        return _frame_dict(r, objs)

    def track_chunk_device(self, bgr, disp, flow, mask, stream=0, parse=True):
        """Device-resident chunk (torch tensors on this context's device, frame-major):
        bgr [F,H,W,3] u8, disp [F,H,W] i16/u16 bits, flow [F,H,W,2] f32, mask [F,H,W] i32.
        parse=False returns the raw (MmtFrameResult[F], MmtMotion[F * MAX_OBJECTS]) arrays."""
        for t, shp in ((bgr, 3), (disp, None), (flow, 2), (mask, None)):
            assert t.is_cuda and t.is_contiguous() and t.shape[1:3] == (self.cfg.height,
                                                                         self.cfg.width)
            assert shp is None or t.shape[3] == shp
        nf = int(bgr.shape[0])
        res = (MmtFrameResult * nf)()
        objs = (MmtMotion * (nf * MAX_OBJECTS))()

        def pitch(t):
            return t.stride(0) * t.element_size()
        self._check(lib().mmt_track_rgbd_chunk_device(
            self._h, nf, bgr.data_ptr(), pitch(bgr), disp.data_ptr(), pitch(disp),
            flow.data_ptr(), pitch(flow), mask.data_ptr(), pitch(mask), res, objs, MAX_OBJECTS,
            ctypes.c_void_p(stream)))
        if not parse:
            return res, objs
        return [_frame_dict(res[i], objs[i * MAX_OBJECTS:(i + 1) * MAX_OBJECTS])
                for i in range(nf)]

    def profile_enable(self, on=True):
        self._check(lib().mmt_profile_enable(self._h, int(on)))

    def profile_read(self, reset=False):
        p = MmtProfile()
        self._check(lib().mmt_profile_read(self._h, ctypes.byref(p), int(reset)))
        return dict(orb_ms=p.orb_ms, orb_launches=p.orb_launches, orb_frames=p.orb_frames)

    # -- probes of single solves ------------------------------------------------------------
    def flow_solve(self, obs, flow, depth, tcw_last, init, rp_thres, prior_info, max_iters,
                   K, use_noise=False, g0=0.0):
        obs = np.ascontiguousarray(obs, np.float32)
        flow = np.ascontiguousarray(flow, np.float32)
        depth = np.ascontiguousarray(depth, np.float32)
        pr = MmtFlowProblem()
        pr.n = len(depth)
        pr.obs, pr.flow, pr.depth = obs.ctypes.data, flow.ctypes.data, depth.ctypes.data
        pr.Tcw_last[:] = np.asarray(tcw_last, np.float32).reshape(16).tolist()
        pr.init[:] = np.asarray(init, np.float32).reshape(16).tolist()
        pr.rp_thres, pr.prior_info, pr.max_iters = rp_thres, prior_info, max_iters
        pr.use_noise, pr.g0 = int(use_noise), g0
        pr.fx, pr.fy, pr.cx, pr.cy = K
        pose = np.zeros(16, np.float32)
        st = np.zeros(3, np.int32)
        self._check(lib().mmt_pose_flow_solve(self._h, ctypes.byref(pr), _p(pose), _p(st)))
        return int(st[2]), pose.reshape(4, 4), dict(iterations=int(st[0]), inliers=int(st[1]))

    def pose_optimization(self, Xw, obs, inv_sigma2, tcw, K, bf):
        """Optimizer::PoseOptimization (D1): (n_inliers, pose 4x4, mvbOutlier flags)."""
        Xw = np.ascontiguousarray(Xw, np.float32)
        obs = np.ascontiguousarray(obs, np.float32)
        s2 = np.ascontiguousarray(inv_sigma2, np.float32)
        n = len(Xw)
        pr = MmtPoseOptProblem()
        pr.n = n
        pr.Xw, pr.obs, pr.inv_sigma2 = Xw.ctypes.data, obs.ctypes.data, s2.ctypes.data
        pr.Tcw[:] = np.asarray(tcw, np.float32).reshape(16).tolist()
        pr.fx, pr.fy, pr.cx, pr.cy = K
        pr.bf = bf
        pose = np.zeros(16, np.float32)
        out = np.zeros(max(n, 1), np.uint8)
        ninl = ctypes.c_int(0)
        self._check(lib().mmt_pose_optimization(self._h, ctypes.byref(pr), _p(pose), _p(out),
                                                ctypes.byref(ninl)))
        return ninl.value, pose.reshape(4, 4), out[:n].astype(bool)

    # ---- B3 / C1-C3 probes (Frame grid, ORBmatcher::SearchByProjection) -------------------
    @staticmethod
    def _match_frame(kps, desc, depth, tcw, keep):
        kps = np.ascontiguousarray(kps)
        desc = np.ascontiguousarray(desc, np.uint8) if desc is not None else None
        depth = np.ascontiguousarray(depth, np.float32)
        keep += [kps, desc, depth]
        fr = MmtMatchFrame()
        fr.n = len(kps)
        fr.kps = kps.ctypes.data
        fr.desc = desc.ctypes.data if desc is not None else None
        fr.depth = depth.ctypes.data
        fr.Tcw[:] = np.asarray(tcw, np.float32).reshape(16).tolist()
        return fr

    def frame_grid(self, kps, depth):
        """Frame::ComputeStereoFromRGBD + AssignFeaturesToGrid (B3): (uR, depth, cell_start,
        cell_idx) with the 64x48 grid as CSR over cells ix*48+iy."""
        keep = []
        fr = self._match_frame(kps, None, depth, np.eye(4), keep)
        n = fr.n
        uR = np.zeros(max(n, 1), np.float32)
        dep = np.zeros(max(n, 1), np.float32)
        cs = np.zeros(64 * 48 + 1, np.int32)
        ci = np.zeros(max(n, 1), np.int32)
        self._check(lib().mmt_frame_grid(self._h, ctypes.byref(fr), _p(uR), _p(dep), _p(cs),
                                         _p(ci)))
        return uR[:n], dep[:n], cs, ci[:cs[-1]]

    def search_by_projection_frame(self, kps, desc, depth, tcw, last_kps, Xw, mp_desc, active,
                                   tlw, th, mono=False, check_orientation=True, obs=None):
        """ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono) (C2):
        (nmatches, match[cur key] = last-frame index or -1).  obs (optional, per last-frame
        point): the point has observations (False: a temporal VO point, whose binding a later
        point may replace)."""
        keep = []
        fr = self._match_frame(kps, desc, depth, tcw, keep)
        lk = np.ascontiguousarray(last_kps)
        X = np.ascontiguousarray(Xw, np.float32)
        md = np.ascontiguousarray(mp_desc, np.uint8)
        act = np.ascontiguousarray(active, np.uint8)
        L = MmtLastFrame()
        L.n = len(lk)
        L.kps, L.Xw, L.mp_desc, L.active = (lk.ctypes.data, X.ctypes.data, md.ctypes.data,
                                            act.ctypes.data)
        L.Tcw[:] = np.asarray(tlw, np.float32).reshape(16).tolist()
        if obs is not None:
            ob = np.ascontiguousarray(obs, np.uint8)
            keep.append(ob)
            L.obs = ob.ctypes.data
        match = np.zeros(max(fr.n, 1), np.int32)
        nm = ctypes.c_int(0)
        self._check(lib().mmt_search_by_projection_frame(
            self._h, ctypes.byref(fr), ctypes.byref(L), th, int(mono), int(check_orientation),
            _p(match), ctypes.byref(nm)))
        return nm.value, match[:fr.n]

    def search_by_bow(self, kf_fv, kf_kps, kf_desc, kf_mp_ok, f_fv, f_kps, f_desc, nnratio=0.7,
                      check_orientation=True):
        """ORBmatcher(nnratio, check_orientation)::SearchByBoW(KeyFrame*, Frame&) (C4):
        (nmatches, match[frame key] = keyframe key or -1).  Feature vectors are (node ids
        ascending, starts, features)."""
        keep = []
        kk = np.ascontiguousarray(kf_kps)
        kd = np.ascontiguousarray(kf_desc, np.uint8)
        ok = np.ascontiguousarray(kf_mp_ok, np.uint8)
        fk = np.ascontiguousarray(f_kps)
        fd = np.ascontiguousarray(f_desc, np.uint8)
        K = MmtBowKeyFrame()
        K.n = len(kk)
        K.kps, K.desc, K.mp_valid = kk.ctypes.data, kd.ctypes.data, ok.ctypes.data
        K.fv = _feature_vector(kf_fv, keep)
        F = _feature_vector(f_fv, keep)
        match = np.zeros(max(len(fk), 1), np.int32)
        nm = ctypes.c_int(0)
        self._check(lib().mmt_search_by_bow(self._h, ctypes.byref(K), len(fk), _p(fk), _p(fd),
                                            ctypes.byref(F), nnratio, int(check_orientation),
                                            _p(match), ctypes.byref(nm)))
        return nm.value, match[:len(fk)]

    def search_local_points(self, kps, desc, depth, tcw, Xw, normal, min_dist, max_dist, pdesc,
                            skip, th, taken=None):
        """Tracking::SearchLocalPoints' isInFrustum pass + ORBmatcher::SearchByProjection(Frame&,
        vector<MapPoint*>, th) (C3): (nmatches, match[cur key], frustum m x 6)."""
        keep = []
        fr = self._match_frame(kps, desc, depth, tcw, keep)
        arrs = [np.ascontiguousarray(a, np.float32) for a in (Xw, normal, min_dist, max_dist)]
        pd = np.ascontiguousarray(pdesc, np.uint8)
        sk = np.ascontiguousarray(skip, np.uint8)
        P = MmtLocalPoints()
        P.m = len(sk)
        P.Xw, P.normal, P.min_dist, P.max_dist = [a.ctypes.data for a in arrs]
        P.desc, P.skip = pd.ctypes.data, sk.ctypes.data
        tk = None if taken is None else np.ascontiguousarray(taken, np.uint8)
        match = np.zeros(max(fr.n, 1), np.int32)
        frus = np.zeros((max(P.m, 1), 6), np.float32)
        nm = ctypes.c_int(0)
        self._check(lib().mmt_search_local_points(
            self._h, ctypes.byref(fr), ctypes.byref(P), th,
            tk.ctypes.data if tk is not None else None, _p(match), _p(frus), ctypes.byref(nm)))
        return nm.value, match[:fr.n], frus[:P.m]

    def fuse_candidates(self, kps, desc, depth, tcw, Xw, normal, min_dist, max_dist, pdesc,
                        th=3.0):
        """ORBmatcher::Fuse(pKF, vpMapPoints, th)'s per-point search against the keyframe (kps,
        desc, depth, tcw): (best key index, best distance) per point, -1 / 256 for none."""
        keep = []
        fr = self._match_frame(kps, desc, depth, tcw, keep)
        arrs = [np.ascontiguousarray(a, np.float32) for a in (Xw, normal, min_dist, max_dist)]
        pd = np.ascontiguousarray(pdesc, np.uint8)
        m = len(arrs[2])
        sk = np.zeros(max(m, 1), np.uint8)
        P = MmtLocalPoints()
        P.m = m
        P.Xw, P.normal, P.min_dist, P.max_dist = [a.ctypes.data for a in arrs]
        P.desc, P.skip = pd.ctypes.data, sk.ctypes.data
        idx = np.zeros(max(m, 1), np.int32)
        dist = np.zeros(max(m, 1), np.int32)
        self._check(lib().mmt_fuse_candidates(self._h, ctypes.byref(fr), ctypes.byref(P),
                                              ctypes.c_float(th), _p(idx), _p(dist)))
        return idx[:m], dist[:m]

    def local_bundle_adjustment(self, P):
        """Optimizer::LocalBundleAdjustment's solve on a problem dict (keys T, fixed, X, pt, kf,
        obs, s, as oracle.Tracker.captured_ba): (T (n_kf, 4, 4), X (n_pt, 3), erase (n_edge,),
        stats dict) like oracle.local_ba."""
        T = np.ascontiguousarray(P["T"], np.float32)
        fx = np.ascontiguousarray(P["fixed"], np.uint8)
        X = np.ascontiguousarray(P["X"], np.float32)
        ept = np.ascontiguousarray(P["pt"], np.int32)
        ekf = np.ascontiguousarray(P["kf"], np.int32)
        eo = np.ascontiguousarray(P["obs"], np.float32)
        es = np.ascontiguousarray(P["s"], np.float32)
        nk, npt, ne = len(fx), len(X), len(ept)
        B = MmtBAProblem(nk, npt, ne, T.ctypes.data, fx.ctypes.data, X.ctypes.data,
                         ept.ctypes.data, ekf.ctypes.data, eo.ctypes.data, es.ctypes.data)
        To = np.zeros((max(nk, 1), 4, 4), np.float32)
        Xo = np.zeros((max(npt, 1), 3), np.float32)
        er = np.zeros(max(ne, 1), np.uint8)
        st = np.zeros(5, np.int32)
        self._check(lib().mmt_local_bundle_adjustment(self._h, ctypes.byref(B), _p(To), _p(Xo),
                                                      _p(er), _p(st)))
        return To[:nk], Xo[:npt], er[:ne], dict(iterations=(int(st[0]), int(st[1])),
                                                 trials=(int(st[2]), int(st[3])),
                                                 n_erase=int(st[4]))

    def set_deferred_objects(self, on=True):
        """mmt_set_deferred_objects: frames return at once, object motions when they are ready
        (each result's objects / objects_frame)."""
        self._check(lib().mmt_set_deferred_objects(self._h, 1 if on else 0))

    def flush_objects(self):
        """mmt_flush_objects until empty: [(objects_frame, objects)] in frame order."""
        return self.flush_objects_part(cap=32, until_empty=True)

    def flush_objects_part(self, cap=32, until_empty=False):
        """One mmt_flush_objects call with res_cap = cap (or calls until none remain)."""
        out = []
        while True:
            res = (MmtFrameResult * cap)()
            objs = (MmtMotion * (cap * MAX_OBJECTS))()
            n = ctypes.c_int(0)
            self._check(lib().mmt_flush_objects(self._h, res, objs, MAX_OBJECTS, cap,
                                                ctypes.byref(n)))
            if n.value == 0:
                return out
            for i in range(n.value):
                d = _frame_dict(res[i], objs[i * MAX_OBJECTS:(i + 1) * MAX_OBJECTS])
                out.append((d["objects_frame"], d["objects"]))
            if not until_empty:
                return out

    def set_keyframe_culling_ratio(self, ratio):
        """Test knob: KeyFrameCulling's redundancy ratio (0.9 in the reference)."""
        self._check(lib().mmt_set_keyframe_culling_ratio(self._h, float(ratio)))

    def map_dump(self):
        """The tracker's map as flat arrays (mmt_map_dump): keyframes (id, frame, bad, parent)
        and poses, each keyframe's map-point slots (CSR), points (position, min/max distance;
        bad, nObs, refKF, firstKFid, replaced), observations (CSR: keyframe, key index, octave;
        key x, y, depth, uR), connections, ordered covisibles (keyframe, other, weight) and
        spanning-tree children (keyframe, child)."""
        sz = np.zeros(7, np.int32)
        self._check(lib().mmt_map_dump(self._h, _p(sz), None))
        out, keep, st = map_dump_arrays(sz)
        self._check(lib().mmt_map_dump(self._h, _p(sz), ctypes.byref(st)))
        del keep
        return out

    def load_vocabulary(self, path):
        """System(voc, ...): DBoW2 text vocabulary; with it the tracker runs the reference's
        TrackReferenceKeyFrame, Relocalization and CreateNewMapPoints (mmt_load_vocabulary)."""
        self._check(lib().mmt_load_vocabulary(self._h, path.encode()))

    def bow_transform(self, desc, levelsup=4):
        """Per descriptor (word, weight, node at level L - levelsup) on the GPU."""
        desc = np.ascontiguousarray(desc, np.uint8)
        n = len(desc)
        w = np.zeros(max(n, 1), np.uint32)
        x = np.zeros(max(n, 1), np.float64)
        nd = np.zeros(max(n, 1), np.uint32)
        self._check(lib().mmt_bow_transform(self._h, _p(desc), n, levelsup, _p(w), _p(x),
                                            _p(nd)))
        return w[:n], x[:n], nd[:n]

    def bow_counters(self):
        """Counters of the vocabulary path (mmt_bow_counters_read)."""
        c = MmtBowCounters()
        self._check(lib().mmt_bow_counters_read(self._h, ctypes.byref(c)))
        return {k: int(getattr(c, k)) for k, _ in MmtBowCounters._fields_}

    def map_counters(self):
        """LocalMapping counters of the context's tracker (mmt_map_counters_read)."""
        c = MmtMapCounters()
        self._check(lib().mmt_map_counters_read(self._h, ctypes.byref(c)))
        return {k: getattr(c, k) for k, _ in MmtMapCounters._fields_}

    def pnp_ransac(self, pts3, pts2, K, max_iters=500, reproj=0.3, conf=0.98):
        pts3 = np.ascontiguousarray(pts3, np.float32)
        pts2 = np.ascontiguousarray(pts2, np.float32)
        n = len(pts3)
        R = np.zeros(9)
        t = np.zeros(3)
        inl = np.zeros(max(n, 1), np.int32)
        ninl = ctypes.c_int(0)
        its = np.zeros(2, np.int32)
        self._check(lib().mmt_pnp_ransac(self._h, _p(pts3), _p(pts2), n, K[0], K[1], K[2], K[3],
                                         max_iters, reproj, conf, _p(R), _p(t), _p(inl),
                                         ctypes.byref(ninl), _p(its)))
        return R.reshape(3, 3), t, inl[:ninl.value].copy(), dict(iterations=int(its[0]),
                                                                 best_iter=int(its[1]))

    def pnpsolver_iterate(self, pts3, pts2, sigma2, K, randi, n_iterations=5, state=None,
                          params=(0.99, 10, 300, 4, 0.5, 5.991)):
        """PnPsolver::SetRansacParameters(*params) + iterate(n_iterations) (row D6) with the
        caller's RandomInt draws `randi` (iterations x 4).  state: dict(iterations,
        best_inliers, best_Tcw, best_mask), updated in place (the solver carried across
        calls).  Returns dict(found, no_more, n_inliers, Tcw, mask) like oracle's."""
        pts3 = np.ascontiguousarray(pts3, np.float32)
        pts2 = np.ascontiguousarray(pts2, np.float32)
        s2 = np.ascontiguousarray(sigma2, np.float32)
        n = len(pts3)
        if state is None:
            state = {}
        pr = MmtPnPsolverProblem()
        pr.n = n
        pr.pts3, pr.pts2, pr.sigma2 = pts3.ctypes.data, pts2.ctypes.data, s2.ctypes.data
        pr.fx, pr.fy, pr.cx, pr.cy = K
        (pr.probability, pr.min_inliers, pr.max_iterations, pr.min_set, pr.epsilon,
         pr.th2) = params
        mask_state = np.ascontiguousarray(state.get("best_mask", np.zeros(n, bool)), np.uint8)
        if len(mask_state) < max(n, 1):
            mask_state = np.zeros(max(n, 1), np.uint8)
        st = MmtPnPsolverState()
        st.iterations = state.get("iterations", 0)
        st.best_inliers = state.get("best_inliers", 0)
        st.best_Tcw[:] = np.asarray(state.get("best_Tcw", np.zeros((4, 4))),
                                    np.float32).reshape(16).tolist()
        st.best_mask = mask_state.ctypes.data
        ri = np.ascontiguousarray(randi, np.int32).reshape(-1, 4)
        T = np.zeros(16, np.float32)
        m = np.zeros(max(n, 1), np.uint8)
        nin, found, no_more = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        self._check(lib().mmt_pnpsolver_iterate(self._h, ctypes.byref(pr), _p(ri), len(ri),
                                                n_iterations, ctypes.byref(st), _p(T), _p(m),
                                                ctypes.byref(nin), ctypes.byref(found),
                                                ctypes.byref(no_more)))
        state.update(iterations=st.iterations, best_inliers=st.best_inliers,
                     best_Tcw=np.array(st.best_Tcw[:], np.float32).reshape(4, 4),
                     best_mask=mask_state[:n].astype(bool))
        return dict(found=bool(found.value), no_more=bool(no_more.value),
                    n_inliers=nin.value, Tcw=T.reshape(4, 4), mask=m[:n].astype(bool))

    def orb_device_status(self, stream=0):
        """mmt_orb_device_status: raises MmtError if an ORB launch tripped a device guard."""
        self._check(lib().mmt_orb_device_status(self._h, stream))

    def debug_orb_raise(self, flags):
        self._check(lib().mmt_debug_orb_raise(self._h, flags))

    def debug_fetch(self, what, frame=0, nbytes=1 << 26):
        buf = np.zeros(nbytes, np.uint8)
        n = self._check(lib().mmt_debug_fetch(self._h, what, frame, _p(buf), nbytes))
        return buf[:n].copy()


class ORBextractor:
    """Mirror of ORB_SLAM2::ORBextractor (reference include/ORBextractor.h), HIP-backed.

    The device context is bound to an image size, created on the first call."""

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device_id=0):
        self.nfeatures, self.scaleFactor, self.nlevels = nfeatures, scaleFactor, nlevels
        self.iniThFAST, self.minThFAST = iniThFAST, minThFAST
        self.device_id = device_id
        self._ctx = None
        self._size = None

    def _context(self, w, h):
        if self._size != (w, h):
            c = kitti03_config(w, h, self.nfeatures, 1, self.device_id)
            c.orb_scale_factor, c.orb_nlevels = self.scaleFactor, self.nlevels
            c.orb_ini_th_fast, c.orb_min_th_fast = self.iniThFAST, self.minThFAST
            self._ctx = Context(c)
            self._size = (w, h)
        return self._ctx

    def __call__(self, image, mask=None):
        image = np.asarray(image)
        assert image.dtype == np.uint8 and image.ndim == 2, "image must be CV_8UC1"
        if image.size == 0:
            return np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8)
        return self._context(image.shape[1], image.shape[0]).orb_extract(image)

    def _tables(self):
        # tables do not depend on the image size; use the kitti03 geometry to build them
        return self._context(*(self._size or (1242, 375))).levels()

    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return self.scaleFactor

    def GetScaleFactors(self):
        return list(self._tables()["scale"])

    def GetInverseScaleFactors(self):
        return [np.float32(1.0) / s for s in self._tables()["scale"]]

    def GetScaleSigmaSquares(self):
        return list(self._tables()["sigma2"])

    def GetInverseScaleSigmaSquares(self):
        return [np.float32(1.0) / s for s in self._tables()["sigma2"]]
