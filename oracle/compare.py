"""Frame-by-frame parity of GPU tracking results against the CPU oracle -- TEST INFRASTRUCTURE.

Both sides are the per-frame dicts of multimot_track_amd.Context.track / track_chunk_device and
oracle.Tracker.track (same keys).  The bar (BASELINE.json north_star): SE(3) poses within 1e-4
(max abs over the 4x4 entries), every integer output exact; the object centroid of the speed
evaluation (ObjCentre3D_pre, metres) within 1e-3.  Poses are float32: past ~1 km of travel a
translation entry's own resolution (one float32 ulp, 6.1e-5 m at 512-1024 m, 1.2e-4 m beyond)
reaches the bar, so an entry also passes when it is within POSE_ULPS ulps of the oracle's value;
the record reports the absolute maximum and the worst entry in ulps.  Used by tests/ and by bench.py's CPU leg
(the parity record of the bench's own frames)."""
import numpy as np

POSE_TOL = 1e-4
POSE_ULPS = 4
CENTRE_TOL = 1e-3
FRAME_INT = ("initialized", "n_keys", "n_obj_samples", "ego_inliers")
OBJ_INT = ("label", "sem_label", "n_points", "ransac_inliers", "mm_inliers", "n_solve",
           "n_inliers")
# LM iteration counts: the stop tests compare chi2 values (a chi2 increase, Raul's 1e-3 test), so
# at a converged solve whose trial chi2 moves only in the last bits, the iteration at which they
# fire follows the rounding of the sums, which a parallel reduction cannot reproduce.  A mismatch
# with the solve's pose within the bar is counted as an LM stop flip (lm_stop_flips), not a
# divergence; with the pose outside the bar the pose comparison reports the frame.
FRAME_LM = ("ego_iterations",)
OBJ_LM = ("iterations",)
OBJ_POSE = ("init", "X", "motion")
# A long parity run may hold a few LM stop flips (tests/golden/d3_stop_tie_c5_f28_o7.npz is the
# documented tie: one float32 ulp of the initial pose moves that solve from 5 to 28 iterations);
# more than this budget is a stop-logic change, even when every pose stays within the bar.
def lm_flip_budget(frames):
    """Largest number of LM stop flips a parity run over `frames` frames may hold."""
    return 1 + int(frames) // 200


MAP_INT = ("map_state", "map_matches_mm", "map_inliers_local", "n_keyframes", "n_mappoints",
           "new_keyframe")


def pose_diff(a, b, counts=None):
    """(max abs diff, max diff in float32 ulps of the oracle entry over the entries at or above
    POSE_TOL (0 when none is), max diff over the entries that fail both POSE_TOL and POSE_ULPS)
    of two 4x4 float32 poses.  counts (optional dict): "entries" += 16, "ulp_only" += the entries
    that pass only by the ulp clause (at or above POSE_TOL, within POSE_ULPS ulps)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    ulps = d / np.spacing(np.abs(b)).astype(np.float64)
    big = d >= POSE_TOL
    fail = big & (ulps > POSE_ULPS)
    if counts is not None:
        counts["entries"] = counts.get("entries", 0) + d.size
        counts["ulp_only"] = counts.get("ulp_only", 0) + int((big & ~fail).sum())
    return (float(d.max()), float(ulps[big].max()) if big.any() else 0.0,
            float(d[fail].max()) if fail.any() else 0.0)


def compare_frame(g, o, counts=None):
    """(max pose diff, max centre diff, [integer mismatch descriptions], max pose diff in ulps,
    max diff of entries failing both bars) of one frame; counts as in pose_diff."""
    bad = []
    for k in FRAME_INT + MAP_INT:
        if k in g and k in o and int(g[k]) != int(o[k]):
            bad.append("%s %r != %r" % (k, g[k], o[k]))
    flips = 0
    for k in FRAME_LM:
        if k in g and k in o and int(g[k]) != int(o[k]):
            flips += 1
    pose, ulps, over = pose_diff(g["Tcw"], o["Tcw"], counts)
    pairs = []
    if "Tcw_map" in g and "Tcw_map" in o:
        pairs.append((g["Tcw_map"], o["Tcw_map"]))
    centre = 0.0
    if len(g["objects"]) != len(o["objects"]):
        bad.append("objects %d != %d" % (len(g["objects"]), len(o["objects"])))
    for j, (a, b) in enumerate(zip(g["objects"], o["objects"])):
        for k in OBJ_INT:
            if int(a[k]) != int(b[k]):
                bad.append("object %d %s %r != %r" % (j, k, a[k], b[k]))
        for k in OBJ_LM:
            if int(a[k]) != int(b[k]):
                flips += 1
        for k in OBJ_POSE:
            pairs.append((a[k], b[k]))
        ca, cb = np.asarray(a["centre_pre"], np.float64), np.asarray(b["centre_pre"], np.float64)
        if not np.array_equal(np.isnan(ca), np.isnan(cb)):  # NaN: a solve without points
            bad.append("object %d centre_pre %s != %s" % (j, ca, cb))
        elif not np.isnan(ca).all():
            centre = max(centre, float(np.nanmax(np.abs(ca - cb))))
    for a, b in pairs:
        p, u, v = pose_diff(a, b, counts)
        pose, ulps, over = max(pose, p), max(ulps, u), max(over, v)
    if counts is not None:
        counts["lm_stop_flips"] = counts.get("lm_stop_flips", 0) + flips
    return pose, centre, bad, ulps, over


def parity_record(gpu_frames, oracle_frames, first_frame=0):
    """Summary over aligned frame lists: frames compared, max pose / centre diff, number of
    frames with an integer mismatch, the first frame that breaks the bar and why."""
    n = min(len(gpu_frames), len(oracle_frames))
    max_pose = max_centre = max_ulps = 0.0
    nbad = 0
    first = None
    why = None
    counts = {"entries": 0, "ulp_only": 0, "lm_stop_flips": 0}
    first_flip = None
    for i in range(n):
        f0 = counts["lm_stop_flips"]
        p, c, bad, u, over = compare_frame(gpu_frames[i], oracle_frames[i], counts)
        if first_flip is None and counts["lm_stop_flips"] > f0:
            first_flip = first_frame + i
        max_pose = max(max_pose, p)
        max_centre = max(max_centre, c)
        max_ulps = max(max_ulps, u)
        if bad:
            nbad += 1
        if first is None and (bad or over > 0 or c >= CENTRE_TOL):
            first = first_frame + i
            why = "; ".join(bad[:4]) if bad else ("pose diff %.3g" % over if over > 0
                                                  else "centre diff %.3g" % c)
    return {"frames": n, "first_frame": first_frame, "max_pose_diff": max_pose,
            "max_pose_diff_ulps": max_ulps, "max_centre_diff": max_centre,
            "int_mismatch_frames": nbad, "first_divergent_frame": first,
            "first_divergence": why, "pose_tol": POSE_TOL, "pose_tol_ulps": POSE_ULPS,
            "pose_entries": counts["entries"], "pose_entries_ulp_only": counts["ulp_only"],
            "lm_stop_flips": counts["lm_stop_flips"], "first_lm_stop_flip": first_flip,
            "centre_tol": CENTRE_TOL}
