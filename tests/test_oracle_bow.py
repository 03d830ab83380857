"""CPU tests of the SearchByBoW oracle (row C4): the C restatement (oracle/match_ref.cpp
search_by_bow) against an independent pure-Python restatement of ORBmatcher::SearchByBoW
(ORBmatcher.cc:532-663) on small synthetic problems, plus hand-built known answers for the
skip-matched rule, the first-of-equal-distances rule, the ratio test and the rotation histogram.
The node assignments are synthetic (ORBvoc.txt is missing): parity given the nodes."""
import numpy as np
import pytest

import bow_problems as BP

POP8 = np.array([bin(i).count("1") for i in range(256)], np.int32)


def hamming(a, b):
    return int(POP8[np.bitwise_xor(a, b)].sum())


def three_maxima(hist):  # ORBmatcher::ComputeThreeMaxima, ORBmatcher.cc:2236-2275
    max1 = max2 = max3 = 0
    i1 = i2 = i3 = -1
    for i, h in enumerate(hist):
        s = len(h)
        if s > max1:
            max3, max2, max1 = max2, max1, s
            i3, i2, i1 = i2, i1, i
        elif s > max2:
            max3, max2 = max2, s
            i3, i2 = i2, i
        elif s > max3:
            max3, i3 = s, i
    if max2 < np.float32(0.1) * np.float32(max1):
        i2 = i3 = -1
    elif max3 < np.float32(0.1) * np.float32(max1):
        i3 = -1
    return i1, i2, i3


def py_search_by_bow(kf_fv, kf_kps, kf_desc, ok, f_fv, f_kps, f_desc, ratio=0.7, orient=True):
    kn, ks, kfeat = kf_fv
    fn, fs, ffeat = f_fv
    match = [-1] * len(f_kps)
    hist = [[] for _ in range(30)]
    nm = 0
    ratio = np.float32(ratio)
    kfn = {int(n): k for k, n in enumerate(kn)}
    for fi, nid in enumerate(fn):  # common nodes, ascending (the merge walk visits each once)
        if int(nid) not in kfn:
            continue
        ki = kfn[int(nid)]
        for a in range(ks[ki], ks[ki + 1]):
            ik = int(kfeat[a])
            if not ok[ik]:
                continue
            b1, b2, bi = 256, 256, -1
            for b in range(fs[fi], fs[fi + 1]):
                jf = int(ffeat[b])
                if match[jf] >= 0:
                    continue
                d = hamming(kf_desc[ik], f_desc[jf])
                if d < b1:
                    b2, b1, bi = b1, d, jf
                elif d < b2:
                    b2 = d
            if b1 <= 50 and np.float32(b1) < ratio * np.float32(b2):
                match[bi] = ik
                if orient:
                    rot = np.float32(kf_kps["angle"][ik]) - np.float32(f_kps["angle"][bi])
                    if rot < 0:
                        rot = np.float32(rot + np.float32(360.0))
                    x = float(np.float32(rot * np.float32(1.0 / 30)))
                    b = int(np.floor(x + 0.5))  # round() half away from zero (x >= 0)
                    if b == 30:
                        b = 0
                    hist[b].append(bi)
                nm += 1
    if orient:
        i1, i2, i3 = three_maxima(hist)
        for i in range(30):
            if i in (i1, i2, i3):
                continue
            for j in hist[i]:
                match[j] = -1
                nm -= 1
    return nm, np.asarray(match, np.int32)


@pytest.mark.parametrize("seed,shuffle,orient", [(0, False, True), (1, True, True),
                                                 (2, False, False), (3, True, False)])
def test_oracle_search_by_bow_matches_python(oracle_mod, seed, shuffle, orient):
    pr = BP.bow_problem(seed, n_kf=150, n_f=200, n_nodes=12, shuffle=shuffle)
    nm_o, m_o = oracle_mod.search_by_bow(*pr, nnratio=0.7, check_orientation=orient)
    nm_p, m_p = py_search_by_bow(*pr, ratio=0.7, orient=orient)
    assert nm_o == nm_p
    assert np.array_equal(m_o, m_p)
    assert nm_o > 10


def _kp(n, angles):
    k = np.zeros(n, BP.KP_DTYPE)
    k["angle"] = angles
    return k


def test_oracle_search_by_bow_known_answers(oracle_mod):
    rng = np.random.default_rng(5)
    d = rng.integers(0, 256, (4, 32), dtype=np.uint8)
    kf_desc = d.copy()
    # frame: key 0 = kf 0 exactly, key 1 = kf 0 exactly too (tie: kf 0 takes key 0, the first of
    # equal distances, and its ratio test 0 < 0.7 * 0 fails -> no match at all), key 2 = kf 1,
    # key 3 = kf 2 with 60 flipped bits (beyond TH_LOW)
    f_desc = np.stack([d[0], d[0], d[1], d[2]])
    f_desc[3, :8] ^= 0xFF
    f_desc[3, 8] ^= 0x0F
    kf_kps = _kp(4, [10, 20, 30, 40])
    f_kps = _kp(4, [10, 10, 20, 30])
    ok = np.ones(4, np.uint8)
    one = (np.array([7], np.uint32), np.array([0, 4], np.int32), np.arange(4, dtype=np.int32))
    nm, m = oracle_mod.search_by_bow(one, kf_kps, kf_desc, ok, one, f_kps, f_desc, 0.7, False)
    assert nm == 1 and m.tolist() == [-1, -1, 1, -1]
    # kf 0 without a MapPoint: kf 1 matches key 2; nothing else
    ok2 = ok.copy()
    ok2[0] = 0
    nm, m = oracle_mod.search_by_bow(one, kf_kps, kf_desc, ok2, one, f_kps, f_desc, 0.7, False)
    assert nm == 1 and m.tolist() == [-1, -1, 1, -1]
    # frame key 1 moved to another node: kf 0 now takes key 0 (second best = 256)
    fv = (np.array([7, 9], np.uint32), np.array([0, 3, 4], np.int32),
          np.array([0, 2, 3, 1], np.int32))
    nm, m = oracle_mod.search_by_bow(one, kf_kps, kf_desc, ok, fv, f_kps, f_desc, 0.7, False)
    assert nm == 2 and m.tolist() == [0, -1, 1, -1]
    # no common node
    other = (np.array([3], np.uint32), np.array([0, 4], np.int32), np.arange(4, dtype=np.int32))
    nm, m = oracle_mod.search_by_bow(one, kf_kps, kf_desc, ok, other, f_kps, f_desc, 0.7, True)
    assert nm == 0 and (m == -1).all()


def test_oracle_search_by_bow_rotation_histogram(oracle_mod):
    # 25 matches rotated by 12 deg (bin round(12/30) = 0), 2 by 300 deg (bin 10): 2 < 0.1 * 25,
    # so only the top bin survives (with 20 + 2 the second bin would stay: 2 < 2.0 is false)
    n = 27
    rng = np.random.default_rng(9)
    d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    ang = rng.uniform(0, 360, n).astype(np.float32)
    fa = (ang - 12) % 360
    fa[-2:] = (ang[-2:] - 300) % 360
    kf_kps, f_kps = _kp(n, ang), _kp(n, fa.astype(np.float32))
    fv = (np.arange(n, dtype=np.uint32), np.arange(n + 1, dtype=np.int32),
          np.arange(n, dtype=np.int32))
    nm, m = oracle_mod.search_by_bow(fv, kf_kps, d, np.ones(n, np.uint8), fv, f_kps, d.copy(),
                                     0.7, True)
    assert nm == 25 and m[:25].tolist() == list(range(25)) and m[25:].tolist() == [-1, -1]
    keep = np.ones(n, bool)
    keep[:5] = False  # 20 + 2: both bins survive
    fv2 = (np.arange(22, dtype=np.uint32), np.arange(23, dtype=np.int32),
           np.nonzero(keep)[0].astype(np.int32))
    nm, m = oracle_mod.search_by_bow(fv2, kf_kps, d, np.ones(n, np.uint8), fv2, f_kps, d.copy(),
                                     0.7, True)
    assert nm == 22 and (m[5:] == np.arange(5, n)).all()
