"""Structural invariants of an ORB-SLAM2 map, checked from scratch on a flat map dump (the
oracle's oracle_tracker_map_dump or the product's mmt_map_dump, same layout).

Written independently of both implementations (which restate MapPoint / KeyFrame bookkeeping
line by line): a misreading shared by the two would pass their parity tests, but not these
checks of what the reference's data structures must satisfy after every LocalMapping:
  * observations <-> keyframe slots: a good point's mObservations entry (kf, i) has
    kf.mvpMapPoints[i] == the point (KeyFrame::AddMapPoint / MapPoint::AddObservation always
    go together, MapPoint.cc:98-137, KeyFrame.cc:188-216), and a good keyframe's slot holding a
    good point belongs to a keyframe the point observes (not necessarily at that slot: a frame
    can hold one point at two keys after CheckReplacedInLastFrame, and ProcessNewKeyFrame then
    keeps the second slot without an observation, LocalMapping.cc:149-166; and two points
    CreateNewMapPoints made from one keyframe-2 feature both observe its slot, which holds the
    second, or nothing once the second went bad);
  * nObs == the recount (2 per observation with mvuRight >= 0, else 1; MapPoint.cc:98-137);
  * mpRefKF is an observer (MapPoint::EraseObservation moves it, MapPoint.cc:111-137);
  * no good point observes a bad keyframe (KeyFrame::SetBadFlag erases its observations,
    KeyFrame.cc:453-470);
  * covisibility: mvpOrderedConnectedKeyFrames is a sub-list of mConnectedKeyFrameWeights with
    the same weights, in non-increasing weight order (KeyFrame.cc:97-115, 218-280); the newest
    keyframe's weights are the from-scratch recount of shared good points as UpdateConnections
    left them, less only the observations its local BA erased afterwards (so never below the
    recount);
  * spanning tree: every good keyframe but the first has a good parent that lists it among
    its children, children name their parent, and parent links reach keyframe 0 without a
    cycle (KeyFrame::ChangeParent / SetBadFlag's re-parenting, KeyFrame.cc:453-545).
Test infrastructure only."""
import numpy as np


def check_map(D, newest=None, cnmp=False):
    """List of violation strings (empty: every invariant holds).  newest: the keyframe whose
    LocalMapping just ran (its covisibility weights are compared with the recount).  cnmp: the
    map comes from a run with CreateNewMapPoints (a vocabulary), whose duplicate slot bindings
    (below) are allowed."""
    bad = []
    kf_i, pt_i = D["kf_i"], D["pt_i"]
    nk, npt = len(kf_i), len(pt_i)
    kbad = kf_i[:, 2].astype(bool)
    ks, slots = D["kf_mps_start"].astype(np.int64), D["kf_mps"]
    os_, oi, of = D["obs_start"], D["obs_i"], D["obs_f"]
    pid = np.repeat(np.arange(npt), np.diff(os_))          # point of each observation
    pgood = pt_i[:, 0] == 0
    og = pgood[pid]                                        # observations of good points
    okf, oidx = oi[:, 0].astype(np.int64), oi[:, 1].astype(np.int64)
    for o in np.nonzero(og & kbad[okf])[0][:20]:
        bad.append("point %d observes bad keyframe %d" % (pid[o], okf[o]))
    held = slots[ks[okf] + oidx]
    # one exception: SearchForTriangulation never sets vbMatched2 (ORBmatcher.cc:1032-1198), so two
    # keyframe-1 features can take the same keyframe-2 feature, and CreateNewMapPoints'
    # AddMapPoint(pMP, idx2) then gives the slot to the second new point while the first keeps its
    # observation (LocalMapping.cc:430-440): the slot's holder observes the same (kf, key)
    key = (pid.astype(np.int64) * nk + okf) * np.int64(1 << 20) + oidx
    keys = set(key[og].tolist())
    for o in np.nonzero(og & (held != pid))[0]:
        if cnmp and held[o] >= 0 and \
                ((int(held[o]) * nk + int(okf[o])) * (1 << 20) + int(oidx[o])) in keys:
            continue
        # ... and once that holder goes bad, SetBadFlag empties the slot (EraseMapPointMatch) while
        # the first point still observes it
        if cnmp and held[o] < 0:
            continue
        bad.append("point %d obs (kf %d, key %d) but the slot holds %d"
                   % (pid[o], okf[o], oidx[o], held[o]))
        if len(bad) >= 20:
            break
    nobs = np.bincount(pid, weights=np.where(of[:, 3] >= 0, 2, 1), minlength=npt)
    for j in np.nonzero(pgood & (nobs != pt_i[:, 1]))[0][:20]:
        bad.append("point %d nObs %d != recount %d" % (j, pt_i[j, 1], nobs[j]))
    isref = np.bincount(pid, weights=(okf == pt_i[pid, 2]), minlength=npt) > 0
    for j in np.nonzero(pgood & (np.diff(os_) > 0) & ~isref)[0][:20]:
        bad.append("point %d refKF %d is not an observer %s"
                   % (j, pt_i[j, 2], okf[os_[j]:os_[j + 1]].tolist()))
    # keyframe slots -> observations
    skf = np.repeat(np.arange(nk), np.diff(ks))
    sidx = np.arange(len(slots)) - ks[skf]
    sel = (slots >= 0) & ~kbad[skf]
    sel[sel] &= pgood[slots[sel]]
    have = np.unique(pid[og] * np.int64(nk) + okf[og])
    want = slots[sel].astype(np.int64) * nk + skf[sel]
    miss = ~np.isin(want, have)
    for q in np.nonzero(miss)[0][:20]:
        bad.append("keyframe %d slot %d holds point %d, which does not observe it"
                   % (skf[sel][q], sidx[sel][q], slots[sel][q]))
    # covisibility
    conn = {}
    for k, q, w in D["conn"]:
        conn.setdefault(int(k), {})[int(q)] = int(w)
    ordl = {}
    for k, q, w in D["ord"]:
        ordl.setdefault(int(k), []).append((int(q), int(w)))
    for k, lst in ordl.items():
        if kbad[k]:
            continue
        ws = [w for _, w in lst]
        if any(ws[i] < ws[i + 1] for i in range(len(ws) - 1)):
            bad.append("keyframe %d ordered covisibles not sorted: %s" % (k, ws))
        for q, w in lst:
            if conn.get(k, {}).get(q) != w:
                bad.append("keyframe %d ordered (%d, %d) not in its weights" % (k, q, w))
    if newest is not None and not kbad[newest]:
        # UpdateConnections' counter from scratch: good points observing the newest keyframe,
        # counted once per other good keyframe they are observed in
        mine = np.zeros(npt, bool)
        mine[pid[og & (okf == newest)]] = True
        m = og & mine[pid] & (okf != newest) & ~kbad[okf]
        pairs = np.unique(pid[m] * np.int64(nk) + okf[m])
        shared = np.bincount(pairs % nk, minlength=nk)
        c = conn.get(newest, {})
        for q in range(nk):
            if kbad[q] or q == newest:
                continue
            if shared[q] > 0 and q not in c:
                bad.append("newest keyframe %d shares %d points with %d but has no weight"
                           % (newest, shared[q], q))
            elif q in c and c[q] < shared[q]:
                bad.append("newest keyframe %d weight to %d is %d < recount %d"
                           % (newest, q, c[q], shared[q]))
    # spanning tree
    children = {}
    for k, ch in D["child"]:
        children.setdefault(int(k), set()).add(int(ch))
    for k in range(nk):
        if kbad[k] or kf_i[k, 0] == 0:
            continue
        par = int(kf_i[k, 3])
        if par < 0 or kbad[par]:
            bad.append("keyframe %d parent %d is missing or bad" % (k, par))
            continue
        if k not in children.get(par, set()):
            bad.append("keyframe %d is not a child of its parent %d" % (k, par))
        seen, x = set(), k
        while kf_i[x, 0] != 0:
            if x in seen or kf_i[x, 3] < 0:
                bad.append("keyframe %d's parent chain does not reach keyframe 0" % k)
                break
            seen.add(x)
            x = int(kf_i[x, 3])
    for k, cs in children.items():
        if kbad[k]:
            continue
        for ch in cs:
            if not kbad[ch] and int(kf_i[ch, 3]) != k:
                bad.append("keyframe %d lists child %d whose parent is %d" % (k, ch, kf_i[ch, 3]))
    return bad


def same_map(A, B):
    """Exact equality of two map dumps' integer structure (keyframes, slots, observations,
    covisibility, tree) and the largest difference of their float fields."""
    diff = []
    for k in ("kf_i", "kf_mps_start", "kf_mps", "pt_i", "obs_start", "obs_i", "conn", "ord",
              "child"):
        if A[k].shape != B[k].shape or not np.array_equal(A[k], B[k]):
            diff.append(k)
    fmax = 0.0
    for k in ("kf_T", "pt_f", "obs_f"):
        if A[k].shape != B[k].shape:
            diff.append(k)
            continue
        a, b = A[k].astype(np.float64), B[k].astype(np.float64)
        fin = np.isfinite(a) & np.isfinite(b)
        if not np.array_equal(np.isfinite(a), np.isfinite(b)):
            diff.append(k + " (finite)")
        if fin.any():
            fmax = max(fmax, float(np.abs(a[fin] - b[fin]).max()))
    return diff, fmax
