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
