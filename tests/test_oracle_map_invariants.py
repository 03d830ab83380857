"""The oracle's map (oracle/map_ref.cpp, mapping_ref.cpp) against the structural invariants of
tests/map_invariants.py after every LocalMapping (CPU, no GPU): a check written independently of
the oracle's restatement of MapPoint / KeyFrame / LocalMapping bookkeeping."""
import numpy as np
import pytest

from map_invariants import check_map


def _half_res_camera():
    # KITTI-03's camera at half resolution: the map logic is resolution-independent and the
    # CPU renderer is four times faster
    from multimot_track_amd import scene
    K = {k: v * 0.5 for k, v in scene.KITTI03.items()}
    return K, 621, 188


@pytest.mark.parametrize("seed,objects,nframes", [(1003, 3, 70)])
def test_oracle_map_invariants_after_every_local_mapping(oracle_mod, seed, objects, nframes):
    from multimot_track_amd import scene
    K, W, H = _half_res_camera()
    R = scene.SequenceRenderer(scene.StreetScene(objects, seed), W, H, K=K)
    tr = oracle_mod.Tracker(W, H, (K["fx"], K["fy"], K["cx"], K["cy"]), K["bf"], 0, 1000)
    n_kf_checks = 0
    for i in range(nframes):
        b, d, f, m = R.frame(i)
        r = tr.track(b.numpy(), d.numpy().view(np.uint16), f.numpy(), m.numpy())
        assert r["map_state"] == 1, i
        if r["new_keyframe"] or i == 0:
            D = tr.map_dump()
            newest = len(D["kf_i"]) - 1
            v = check_map(D, newest=newest)
            assert v == [], (i, v[:10], len(v))
            n_kf_checks += 1
    st = tr.map_stats()
    assert n_kf_checks > 10 and st["n_ba"] > 8 and st["n_fused"] > 0 and st["n_ba_erased"] > 0


def test_map_invariants_catch_corruption(oracle_mod):
    """The checker is not vacuous: each kind of corruption of a valid map dump is reported."""
    from multimot_track_amd import scene
    K, W, H = _half_res_camera()
    R = scene.SequenceRenderer(scene.StreetScene(3, 1003), W, H, K=K)
    tr = oracle_mod.Tracker(W, H, (K["fx"], K["fy"], K["cx"], K["cy"]), K["bf"], 0, 1000)
    for i in range(12):
        b, d, f, m = R.frame(i)
        tr.track(b.numpy(), d.numpy().view(np.uint16), f.numpy(), m.numpy())
    D = tr.map_dump()
    assert check_map(D) == []
    good = np.nonzero((D["pt_i"][:, 0] == 0) & (np.diff(D["obs_start"]) >= 2))[0]
    j = int(good[0])

    def corrupt(fn):
        E = {k: v.copy() for k, v in D.items()}
        fn(E)
        return check_map(E)
    assert any("nObs" in v for v in corrupt(lambda E: E["pt_i"].__setitem__((j, 1), 99)))
    assert any("refKF" in v for v in corrupt(lambda E: E["pt_i"].__setitem__((j, 2), 10 ** 6)))
    o = D["obs_start"][j]
    k, idx = D["obs_i"][o, :2]
    assert any("slot holds" in v for v in
               corrupt(lambda E: E["kf_mps"].__setitem__(E["kf_mps_start"][k] + idx, -1)))
    kk = int(np.nonzero(D["kf_i"][:, 0] > 0)[0][-1])
    assert any("parent" in v for v in corrupt(lambda E: E["kf_i"].__setitem__((kk, 3), kk)))
    assert any("sorted" in v or "not in its weights" in v for v in
               corrupt(lambda E: E["ord"].__setitem__((0, 2), E["ord"][0, 2] + 1000)))


def test_oracle_relocalization_recovers_after_lost_frame(oracle_mod):
    """A frame without texture (no ORB keys) loses map tracking; the relocalization substitute
    (oracle/map_ref.cpp relocalization_subst: the reference keyframe's and its covisibles' map
    points at the motion model's prediction, the reference's acceptance tests) recovers on the
    next frame, and the map passes the invariant checks after it."""
    from multimot_track_amd import scene
    K, W, H = _half_res_camera()
    R = scene.SequenceRenderer(scene.StreetScene(3, 1003), W, H, K=K)
    tr = oracle_mod.Tracker(W, H, (K["fx"], K["fy"], K["cx"], K["cy"]), K["bf"], 0, 1000)
    states = []
    for i in range(43):
        b, d, f, m = R.frame(i)
        b = b.numpy()
        if i == 40:
            b = np.full_like(b, 128)
        r = tr.track(b, d.numpy().view(np.uint16), f.numpy(), m.numpy())
        states.append(r["map_state"])
    assert states[:40] == [1] * 40 and states[40] == 2 and states[41:] == [1, 1]
    assert check_map(tr.map_dump()) == []


def test_oracle_keyframe_culling_reparents_and_keeps_invariants(oracle_mod):
    """KeyFrameCulling (LocalMapping.cc:653-720) with KeyFrame::SetBadFlag's re-parenting
    (KeyFrame.cc:453-545).  The synthetic sequences never reach the reference's 0.9 redundancy
    ratio, so the test lowers it (the test knob, oracle set_cull_ratio / the product's
    mmt_set_keyframe_culling_ratio) on a slow drive (the GPU test's 3/4-resolution sequence):
    keyframes are culled, spanning-tree children are re-parented, and the map passes every
    invariant after each LocalMapping."""
    from multimot_track_amd import scene
    K = {k: v * 0.75 for k, v in scene.KITTI03.items()}
    W, H = 931, 281
    R = scene.SequenceRenderer(scene.StreetScene(3, 1003, speed=0.3), W, H, K=K)
    tr = oracle_mod.Tracker(W, H, (K["fx"], K["fy"], K["cx"], K["cy"]), K["bf"], 0, 1500)
    tr.set_cull_ratio(0.3)
    for i in range(60):
        b, d, f, m = R.frame(i)
        r = tr.track(b.numpy(), d.numpy().view(np.uint16), f.numpy(), m.numpy())
        assert r["map_state"] == 1, i
        if r["new_keyframe"]:
            D = tr.map_dump()
            assert check_map(D, newest=len(D["kf_i"]) - 1) == [], i
    st = tr.map_stats()
    assert st["n_culled"] >= 2 and st["n_reparent"] >= 1, st
    D = tr.map_dump()
    assert int(D["kf_i"][:, 2].sum()) == st["n_culled"]
