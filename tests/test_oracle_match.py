"""CPU tests of the matching oracle (rows B3, C1-C3): the C restatement (oracle/match_ref.cpp)
against a second, independent pure-Python restatement of the same reference functions
(Frame::ComputeStereoFromRGBD / AssignFeaturesToGrid / GetFeaturesInArea / isInFrustum,
MapPoint::PredictScale, ORBmatcher::SearchByProjection x2, DescriptorDistance), written straight
from the reference text on real kitti_sample keypoints.  The reference ships no golden vectors
for these functions: parity with OpenCV/ORB-SLAM2 builds is unpinned, see DESIGN.md."""
import math

import numpy as np
import pytest

import match_problems as MP

f32 = np.float32
POP8 = np.array([bin(i).count("1") for i in range(256)], np.int32)


def hamming(a, b):
    return int(POP8[np.bitwise_xor(a, b)].sum())


def py_grid(kps, depth):
    """ComputeStereoFromRGBD + AssignFeaturesToGrid, Frame.cc:1041-1062, 601-616, 765-775."""
    n = len(kps)
    uR = np.full(n, -1, np.float32)
    dep = np.full(n, -1, np.float32)
    invW = f32(64) / f32(MP.W)
    invH = f32(48) / f32(MP.H)
    grid = [[] for _ in range(64 * 48)]
    for i in range(n):
        x, y = f32(kps["x"][i]), f32(kps["y"][i])
        d = depth[int(y), int(x)]
        if d > 0:
            dep[i] = d
            uR[i] = x - f32(MP.BF) / d
        gx = x * invW
        gy = y * invH
        px = int(math.floor(float(gx) + 0.5)) if gx >= 0 else -int(math.floor(-float(gx) + 0.5))
        py = int(math.floor(float(gy) + 0.5)) if gy >= 0 else -int(math.floor(-float(gy) + 0.5))
        if 0 <= px < 64 and 0 <= py < 48:
            grid[px * 48 + py].append(i)
    return uR, dep, grid, invW, invH


def py_area(kps, grid, invW, invH, x, y, r, minL, maxL):
    out = []
    if not (math.isfinite(x) and math.isfinite(y)):  # pinned: no cells (see match_ref.cpp)
        return out
    cx0 = max(0, int(math.floor(f32(x - f32(0) - r) * invW)))
    if cx0 >= 64:
        return out
    cx1 = min(63, int(math.ceil(f32(x - f32(0) + r) * invW)))
    if cx1 < 0:
        return out
    cy0 = max(0, int(math.floor(f32(y - f32(0) - r) * invH)))
    if cy0 >= 48:
        return out
    cy1 = min(47, int(math.ceil(f32(y - f32(0) + r) * invH)))
    if cy1 < 0:
        return out
    check = minL > 0 or maxL >= 0
    for ix in range(cx0, cx1 + 1):
        for iy in range(cy0, cy1 + 1):
            for k in grid[ix * 48 + iy]:
                o = kps["octave"][k]
                if check and (o < minL or (maxL >= 0 and o > maxL)):
                    continue
                if abs(f32(kps["x"][k]) - x) < r and abs(f32(kps["y"][k]) - y) < r:
                    out.append(k)
    return out


def xform(T, X):
    R = T[:3, :3].astype(np.float64)
    return [f32(R[r] @ np.asarray(X, np.float64)) + f32(T[r, 3]) for r in range(3)]


def centre(T):
    R = T[:3, :3].astype(np.float64)
    return [f32(-(R[:, r] @ T[:3, 3].astype(np.float64))) for r in range(3)]


def py_sbp_frame(c, scale):
    """ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono), ORBmatcher.cc:1958-2102."""
    kps, desc = c["kps"], c["desc"]
    uR, _, grid, invW, invH = py_grid(kps, c["depth"])
    fx, fy, cx, cy = [f32(v) for v in MP.K]
    bf = f32(MP.BF)
    Tc, Tl = c["tcw"].astype(np.float32), c["tlw"].astype(np.float32)
    tlc = xform(Tl, centre(Tc))
    mb = bf / fx
    fwd = tlc[2] > mb and not c["mono"]
    bwd = -tlc[2] > mb and not c["mono"]
    match = np.full(len(kps), -1, np.int32)
    taken = np.zeros(len(kps), bool)  # bound to a point with observations
    obs = c.get("obs")
    hist = [[] for _ in range(30)]
    nm = 0
    th = f32(c["th"])
    for i in range(len(c["last_kps"])):
        if not c["active"][i]:
            continue
        xc, yc, zc = xform(Tc, c["Xw"][i])
        invz = f32(1.0 / float(zc))
        if invz < 0:
            continue
        u = fx * xc * invz + cx
        v = fy * yc * invz + cy
        if u < 0 or u > f32(MP.W) or v < 0 or v > f32(MP.H):
            continue
        lo = int(c["last_kps"]["octave"][i])
        rad = th * f32(scale[lo])
        if fwd:
            cand = py_area(kps, grid, invW, invH, u, v, rad, lo, -1)
        elif bwd:
            cand = py_area(kps, grid, invW, invH, u, v, rad, 0, lo)
        else:
            cand = py_area(kps, grid, invW, invH, u, v, rad, lo - 1, lo + 1)
        best, bi = 256, -1
        for k in cand:
            if taken[k]:
                continue
            if uR[k] > 0 and abs((u - bf * invz) - uR[k]) > rad:
                continue
            d = hamming(c["mp_desc"][i], desc[k])
            if d < best:
                best, bi = d, k
        if best <= 100:
            match[bi] = i
            taken[bi] = obs is None or bool(obs[i])
            nm += 1
            if c["check_orientation"]:
                rot = f32(c["last_kps"]["angle"][i]) - f32(kps["angle"][bi])
                if rot < 0:
                    rot += f32(360)
                q = float(rot * (f32(1) / f32(30)))
                b = int(math.floor(q + 0.5))
                hist[0 if b == 30 else b].append(bi)
    if c["check_orientation"]:
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for b in range(30):
            s = len(hist[b])
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, b
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, b
            elif s > m3:
                m3, i3 = s, b
        if m2 < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif m3 < f32(0.1) * f32(m1):
            i3 = -1
        for b in range(30):
            if b not in (i1, i2, i3):
                for k in hist[b]:
                    match[k] = -1
                    nm -= 1
    return nm, match


def py_local(c, scale):
    """SearchLocalPoints (Tracking.cc:3416-3466) + SearchByProjection(Frame&, vector<MapPoint*>)."""
    kps, desc = c["kps"], c["desc"]
    uR, _, grid, invW, invH = py_grid(kps, c["depth"])
    fx, fy, cx, cy = [f32(v) for v in MP.K]
    bf = f32(MP.BF)
    T = c["tcw"].astype(np.float32)
    Ow = centre(T)
    logs = f32(math.log(float(f32(1.2))))
    fr = []
    for j in range(len(c["Xw"])):
        rec = None
        if not c["skip"][j]:
            P = c["Xw"][j]
            pc = xform(T, P)
            if not pc[2] < 0:
                invz = f32(1) / pc[2]
                u = fx * pc[0] * invz + cx
                v = fy * pc[1] * invz + cy
                if 0 <= u <= f32(MP.W) and 0 <= v <= f32(MP.H):
                    PO = [f32(P[k]) - Ow[k] for k in range(3)]
                    dist = f32(math.sqrt(sum(float(p) * float(p) for p in PO)))
                    if not (dist < f32(0.8) * c["min_dist"][j] or dist > f32(1.2) * c["max_dist"][j]):
                        dot = sum(float(PO[k]) * float(c["normal"][j][k]) for k in range(3))
                        vc = f32(dot / float(dist))
                        if not vc < f32(0.5):
                            ratio = f32(c["max_dist"][j]) / dist
                            lv = int(math.ceil(f32(math.log(float(ratio))) / logs))
                            lv = min(max(lv, 0), 7)
                            rec = (lv, u, v, u - bf * invz, vc)
        fr.append(rec)
    bound = c["taken"].astype(bool).copy()
    match = np.full(len(kps), -1, np.int32)
    nm = 0
    th = f32(c["th"])
    if not any(r is not None for r in fr):
        return 0, match, fr
    for j, rec in enumerate(fr):
        if rec is None:
            continue
        lv, u, v, ur, vc = rec
        r = f32(2.5) if float(vc) > 0.998 else f32(4.0)
        if th != 1.0:
            r = r * th
        rr = r * f32(scale[lv])
        cand = py_area(kps, grid, invW, invH, u, v, rr, lv - 1, lv)
        b1, l1, b2, l2, bi = 256, -1, 256, -1, -1
        for k in cand:
            if bound[k]:
                continue
            if uR[k] > 0 and abs(ur - uR[k]) > rr:
                continue
            d = hamming(c["pdesc"][j], desc[k])
            if d < b1:
                b2, l2, b1, l1, bi = b1, l1, d, int(kps["octave"][k]), k
            elif d < b2:
                b2, l2 = d, int(kps["octave"][k])
        if b1 <= 100:
            if l1 == l2 and f32(b1) > f32(0.8) * f32(b2):
                continue
            bound[bi] = True
            match[bi] = j
            nm += 1
    return nm, match, fr


def test_grid_matches_python_restatement(oracle_mod):
    k, _, dep = MP.frame(oracle_mod, 1)
    uR, d, cs, ci = oracle_mod.frame_stereo_grid(k, dep, MP.K, MP.BF)
    puR, pd, grid, _, _ = py_grid(k, dep)
    assert np.array_equal(uR, puR) and np.array_equal(d, pd)
    flat = [i for cell in grid for i in cell]
    assert np.array_equal(ci, np.array(flat, np.int32))
    assert np.array_equal(np.diff(cs), [len(cell) for cell in grid])
    assert (uR > 0).sum() > 1000 and len(ci) == len(k)  # every kitti key lands in the grid


@pytest.mark.parametrize("name", MP.SBP_CASES)
def test_search_by_projection_frame_python(oracle_mod, name):
    c = MP.sbp_case(oracle_mod, name)
    scale = MP.scale_factors(oracle_mod)
    nm, match = oracle_mod.search_by_projection_frame(
        c["kps"], c["desc"], c["depth"], c["tcw"], c["last_kps"], c["Xw"], c["mp_desc"],
        c["active"], c["tlw"], c["th"], MP.K, MP.BF, scale, c["mono"], c["check_orientation"],
        obs=c["obs"])
    pnm, pmatch = py_sbp_frame(c, scale)
    assert nm == pnm and np.array_equal(match, pmatch)
    if c["obs"] is None:
        assert nm == (match >= 0).sum()
    else:  # rebinding: nmatches counts every binding, the key keeps its last binder
        assert nm >= (match >= 0).sum()
    if name in ("forward", "backward", "mono_wide", "duplicates", "vo_points", "vo_duplicates"):
        assert nm > 50, nm
    # every bound pair is a real descriptor match within TH_HIGH
    for k in np.nonzero(match >= 0)[0][:200]:
        assert hamming(c["mp_desc"][match[k]], c["desc"][k]) <= 100


@pytest.mark.parametrize("name", MP.LOCAL_CASES)
def test_search_local_points_python(oracle_mod, name):
    c = MP.local_case(oracle_mod, name)
    scale = MP.scale_factors(oracle_mod)
    nm, match, frus = oracle_mod.search_local_points(
        c["kps"], c["desc"], c["depth"], c["tcw"], c["Xw"], c["normal"], c["min_dist"],
        c["max_dist"], c["pdesc"], c["skip"], c["th"], MP.K, MP.BF, scale, c["taken"])
    pnm, pmatch, pfr = py_local(c, scale)
    assert nm == pnm and np.array_equal(match, pmatch)
    inview = np.array([r is not None for r in pfr])
    assert np.array_equal(frus[:, 0].astype(bool), inview)
    lv = np.array([r[0] if r is not None else 0 for r in pfr])
    assert np.array_equal(frus[inview, 1].astype(int), lv[inview])
    assert not np.any((match >= 0) & (c["taken"] != 0))
    assert inview.sum() > 100 and nm > 20, (inview.sum(), nm)
