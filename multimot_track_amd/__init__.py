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
LIB_PATH = os.path.join(_HERE, "libmmt.so")
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
                ("device_id", ctypes.c_int), ("max_batch", ctypes.c_int)]


class MmtError(RuntimeError):
    pass


def lib():
    """Load libmmt.so; fail loudly (no fallback) when the HIP extension is not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise MmtError("libmmt.so not built: run `python -c 'import __graft_entry__ as g; "
                           "g.build()'` (there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
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
        L.mmt_debug_fetch.restype = ctypes.c_long
        L.mmt_debug_fetch.argtypes = [vp, i32, i32, vp, sz]
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
    c.bf, c.th_depth, c.rgb = 387.5744, 65.2, 1
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
        if getattr(self, "_h", None):
            lib().mmt_destroy(self._h)
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
