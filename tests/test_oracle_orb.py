"""CPU tests of the ORB oracle (oracle/orb_ref.cpp): known answers for every in-tree constant of
the reference path, invariants of each pinned OpenCV primitive, and drift detection against the
committed golden fixture tests/golden/orb_kitti.npz (made by tools/make_golden_orb.py)."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN


def test_level_quotas_known_answers(oracle_mod):
    # ORBextractor.cc:436-446 -- values listed in SURVEY.md section 8(a) A5
    assert list(oracle_mod.orb_config(2000)["n_per_level"]) == [434, 362, 302, 251, 209, 175, 145, 122]
    assert list(oracle_mod.orb_config(4000)["n_per_level"]) == [869, 724, 603, 503, 419, 349, 291, 242]
    assert list(oracle_mod.orb_config(8000)["n_per_level"]) == [1737, 1448, 1207, 1005, 838, 698, 582, 485]


def test_umax_known_answer(oracle_mod):
    # ORBextractor.cc:454-469 (the classic ORB circular-patch row extents)
    assert list(oracle_mod.orb_config()["umax"]) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


def test_scale_factors(oracle_mod):
    c = oracle_mod.orb_config()
    s = np.float32(1.0)
    for l in range(8):
        assert c["scale"][l] == s
        s = np.float32(np.float64(s) * np.float64(np.float32(1.2)))


def test_level_sizes_known_answers(oracle_mod):
    # SURVEY.md 8(a) A3 table
    lw, lh = oracle_mod.level_sizes(1242, 375)
    assert list(zip(lw, lh)) == [(1242, 375), (1035, 312), (862, 260), (719, 217), (599, 181),
                                 (499, 151), (416, 126), (347, 105)]
    lw, lh = oracle_mod.level_sizes(1920, 1080)
    assert (lw[-1], lh[-1]) == (536, 301)


def test_gray_weights(oracle_mod):
    # RGB2GRAY applied to BGR memory order: channel 0 (B) gets the R weight 4899 (Appendix A.1)
    img = np.zeros((1, 4, 3), np.uint8)
    img[0, 0] = (255, 0, 0)
    img[0, 1] = (0, 255, 0)
    img[0, 2] = (0, 0, 255)
    img[0, 3] = (10, 20, 30)
    g = oracle_mod.gray_from_bgr(img)[0]
    assert list(g) == [(255 * 4899 + 8192) >> 14, (255 * 9617 + 8192) >> 14,
                       (255 * 1868 + 8192) >> 14, (10 * 4899 + 20 * 9617 + 30 * 1868 + 8192) >> 14]


def test_blur_constant_and_taps(oracle_mod):
    # taps sum to 256 -> a constant image is a fixed point of the Q8/Q16 filter
    img = np.full((40, 50), 173, np.uint8)
    assert (oracle_mod.blur7(img) == 173).all()
    # impulse response = outer product of the ED taps [18,34,48,56,48,34,18]
    img = np.zeros((21, 21), np.uint8)
    img[10, 10] = 255
    out = oracle_mod.blur7(img).astype(np.int64)
    taps = np.array([18, 34, 48, 56, 48, 34, 18], np.int64)
    exp = (np.outer(taps, taps) * 255 + 32768) >> 16
    assert (out[7:14, 7:14] == exp).all()


def test_fast_atan2(oracle_mod):
    assert abs(oracle_mod.fast_atan2(1, 1) - 45.0) < 0.02
    assert abs(oracle_mod.fast_atan2(1, 0) - 90.0) < 1e-4
    assert abs(oracle_mod.fast_atan2(0, -1) - 180.0) < 1e-4
    assert abs(oracle_mod.fast_atan2(-1, 0) - 270.0) < 1e-4
    assert oracle_mod.fast_atan2(0, 0) == 0.0
    for y, x in [(3, 7), (-5, 2), (11, -13), (-1, -1)]:
        ref = np.degrees(np.arctan2(y, x)) % 360
        assert abs(oracle_mod.fast_atan2(y, x) - ref) < 0.02


def test_resize_constant_and_monotone(oracle_mod):
    g = np.full((375, 1242), 99, np.uint8)
    for lev in oracle_mod.pyramid(g):
        assert (lev == 99).all()
    ramp = np.tile(np.arange(1242) % 256, (375, 1)).astype(np.uint8)
    lev1 = oracle_mod.pyramid(ramp, nlevels=2)[1]
    assert (np.diff(lev1[:, :200].astype(int), axis=1) >= 0).all()


def test_fast_constant_image_has_no_keys(oracle_mod):
    g = np.full((200, 300), 50, np.uint8)
    k, d = oracle_mod.orb_extract(g, 500)
    assert len(k) == 0 and d.shape == (0, 32)


def test_octree_invariants(oracle_mod, kitti_frames):
    g = oracle_mod.gray_from_bgr(kitti_frames[0]["bgr"])
    pyr = oracle_mod.pyramid(g)
    for nf in (2000, 8000):
        npl = oracle_mod.orb_config(nf)["n_per_level"]
        for l, im in enumerate(pyr):
            cand = oracle_mod.level_candidates(im)
            h, w = im.shape
            sel = oracle_mod.distribute(cand, 16, w - 16, 16, h - 16, int(npl[l]))
            # a subset of the candidates, at most quota + 3, unique positions
            assert len(sel) <= npl[l] + 3
            cs = {tuple(r) for r in cand.tolist()}
            assert all(tuple(r) in cs for r in sel.tolist())
            assert len({(r[0], r[1]) for r in sel.tolist()}) == len(sel)


def test_extract_shapes_and_levels(oracle_mod, kitti_frames):
    g = oracle_mod.gray_from_bgr(kitti_frames[0]["bgr"])
    k, d = oracle_mod.orb_extract(g, 2000)
    assert d.shape == (len(k), 32)
    assert (np.diff(k["octave"]) >= 0).all()          # level-major output
    assert set(np.unique(k["size"])) <= {31., 37., 44., 53., 64., 77., 92., 111.}
    assert ((k["angle"] >= 0) & (k["angle"] <= 360)).all()


def _digest(k, d):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(k).tobytes())
    h.update(np.ascontiguousarray(d).tobytes())
    return h.hexdigest()


def test_oracle_matches_committed_golden(oracle_mod, kitti_frames):
    path = os.path.join(GOLDEN, "orb_kitti.npz")
    if not os.path.exists(path):
        pytest.skip("golden fixture not generated")
    gold = np.load(path)
    for i, fr in enumerate(kitti_frames):
        g = oracle_mod.gray_from_bgr(fr["bgr"])
        for nf in (2000, 4000):
            k, d = oracle_mod.orb_extract(g, nf)
            assert _digest(k, d) == str(gold["digest_f%d_n%d" % (i, nf)])
    g = oracle_mod.gray_from_bgr(kitti_frames[0]["bgr"])
    k, d = oracle_mod.orb_extract(g, 2000)
    assert np.array_equal(k.view(np.uint8), gold["kps_f0_n2000"].view(np.uint8))
    assert np.array_equal(d, gold["desc_f0_n2000"])
