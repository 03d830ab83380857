"""Synthetic inputs of ORBmatcher::SearchByBoW (C4): a keyframe and a frame whose features carry
caller-supplied DBoW2 FeatureVectors (the vocabulary ORBvoc.txt is missing from the reference, so
node assignments are synthetic: parity of the matcher given the nodes).  Part of the frame
features are bit-flipped copies of keyframe descriptors (some beyond TH_LOW), rotated by a common
angle with a share of rotation outliers, so the ratio test, the matched-feature skip and the
rotation histogram all act."""
import numpy as np

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


def _kps(rng, n):
    k = np.zeros(n, KP_DTYPE)
    k["x"] = rng.uniform(20, 1220, n).astype(np.float32)
    k["y"] = rng.uniform(20, 355, n).astype(np.float32)
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["octave"] = rng.integers(0, 8, n)
    k["size"] = 31
    return k


def feature_vector(nodes, shuffle_rng=None):
    """node id per feature -> (node ids ascending, starts, features): DBoW2 pushes features in
    index order; shuffle_rng permutes each node's list (order-dependence check)."""
    nodes = np.asarray(nodes)
    ids = np.unique(nodes)
    start = [0]
    feat = []
    for nid in ids:
        f = np.nonzero(nodes == nid)[0]
        if shuffle_rng is not None:
            f = shuffle_rng.permutation(f)
        feat.extend(f.tolist())
        start.append(len(feat))
    return (ids.astype(np.uint32), np.asarray(start, np.int32), np.asarray(feat, np.int32))


def bow_problem(seed, n_kf=1500, n_f=2000, n_nodes=120, frac_match=0.6, rot=12.0,
                rot_outliers=0.15, mp_valid=0.85, shuffle=False, dup=0.05):
    rng = np.random.default_rng(seed)
    kf_desc = rng.integers(0, 256, (n_kf, 32), dtype=np.uint8)
    kf_kps = _kps(rng, n_kf)
    kf_nodes = rng.integers(0, n_nodes, n_kf)
    f_desc = rng.integers(0, 256, (n_f, 32), dtype=np.uint8)
    f_kps = _kps(rng, n_f)
    f_nodes = rng.integers(0, n_nodes, n_f)
    m = min(int(frac_match * n_f), n_kf)
    src = rng.permutation(n_kf)[:m]
    for j, s in enumerate(src):
        d = kf_desc[s].copy()
        nflip = int(rng.integers(0, 70))
        bits = rng.choice(256, nflip, replace=False)
        for b in bits:
            d[b // 8] ^= np.uint8(1 << (b % 8))
        f_desc[j] = d
        a = kf_kps["angle"][s] - rot + rng.normal(0, 2.0)
        if rng.uniform() < rot_outliers:
            a = rng.uniform(0, 360)
        f_kps["angle"][j] = np.float32(a % 360.0)
        f_nodes[j] = kf_nodes[s] if rng.uniform() < 0.9 else rng.integers(0, n_nodes)
    # exact duplicates of a matched descriptor: equal distances (first-of-equal and ratio ties)
    nd = int(dup * m)
    for j in range(nd):
        t = m + j
        if t >= n_f:
            break
        f_desc[t] = f_desc[j]
        f_nodes[t] = f_nodes[j]
        f_kps["angle"][t] = f_kps["angle"][j]
    ok = (rng.uniform(size=n_kf) < mp_valid).astype(np.uint8)
    srng = np.random.default_rng(seed + 1000) if shuffle else None
    return (feature_vector(kf_nodes, srng), kf_kps, kf_desc, ok,
            feature_vector(f_nodes, srng), f_kps, f_desc)
