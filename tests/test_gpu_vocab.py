"""GPU parity of the vocabulary-driven path against the CPU oracle.

The DBoW2 vocabulary is tests/golden/test_voc_k10l6.txt (the reference's ORBvoc.txt is missing;
tools/make_test_vocabulary.py writes this one in the same text format).  With it the tracker runs
the reference's TrackReferenceKeyFrame (SearchByBoW against the reference keyframe),
Relocalization (keyframe database, SearchByBoW, PnPsolver, the SearchByProjection(F, KF) rounds)
and LocalMapping's CreateNewMapPoints (SearchForTriangulation), on the GPU kernels of
mmt_bow.hip / mmt_match.hip / mmt_pnp.hip / mmt_lm.hip.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_kitti_frame
from synth_problems import K_KITTI

pytestmark = pytest.mark.gpu

VOC = os.path.join(GOLDEN, "test_voc_k10l6.txt")
BOW_KEYS = ("bow_frames", "trk", "trk_ok", "reloc", "reloc_ok", "reloc_cands", "pnp_found",
            "sbp_rounds", "triangulated", "sft_matches", "kfdb")


def test_bow_transform_bit_exact(oracle_mod):
    """k_bow_transform (one descent per descriptor) against the oracle's transform over the
    kitti_sample frames' descriptors: word ids, weights and level-2 nodes identical."""
    import multimot_track_amd as M
    ov = oracle_mod.Vocabulary(VOC)
    ctx = M.Context(M.kitti03_config(1242, 375, 2000))
    try:
        ctx.load_vocabulary(VOC)
        for i in range(5):
            g = oracle_mod.gray_from_bgr(load_kitti_frame(i)["bgr"])
            _, d = oracle_mod.orb_extract(g, 2000)
            for levelsup in (4, 3, 6):
                w, x, nd = ctx.bow_transform(d, levelsup)
                r = ov.transform(d, levelsup)
                assert np.array_equal(w, r["word"]), (i, levelsup)
                assert np.array_equal(x, r["weight"]), (i, levelsup)
                assert np.array_equal(nd, r["node"]), (i, levelsup)
        # random descriptors (far from every training descriptor: ties at every level)
        d = np.random.default_rng(5).integers(0, 256, (3000, 32), dtype=np.uint8)
        w, x, nd = ctx.bow_transform(d, 4)
        r = ov.transform(d, 4)
        assert np.array_equal(w, r["word"]) and np.array_equal(nd, r["node"])
    finally:
        ctx.close()


def test_load_vocabulary_errors(tmp_path):
    import multimot_track_amd as M
    ctx = M.Context(M.kitti03_config(1242, 375, 2000))
    try:
        with pytest.raises(RuntimeError):
            ctx.load_vocabulary(str(tmp_path / "missing.txt"))
        p = tmp_path / "bad.txt"
        p.write_text("10 12 0 0\n")  # L > 10 (TemplatedVocabulary.h:1359)
        with pytest.raises(RuntimeError):
            ctx.load_vocabulary(str(p))
        ctx.load_vocabulary(VOC)
    finally:
        ctx.close()


def _run_pair(oracle_mod, W, H, K, bf, nfeat, n, lost, chunk=16, seed=1003):
    import torch
    import multimot_track_amd as M
    from multimot_track_amd import scene
    dev = torch.device("cuda:0")
    R = scene.SequenceRenderer(scene.StreetScene(3, seed), W, H, K=K, device=dev)
    seq = R.sequence(n)
    for i in lost:
        seq["bgr"][i] = 128
    cfg = M.kitti03_config(W, H, nfeat, max_batch=chunk)
    cfg.fx, cfg.fy, cfg.cx, cfg.cy, cfg.bf = K["fx"], K["fy"], K["cx"], K["cy"], bf
    ctx = M.Context(cfg)
    got = []
    try:
        ctx.load_vocabulary(VOC)
        for s0 in range(0, n, chunk):
            sl = slice(s0, min(n, s0 + chunk))
            got += ctx.track_chunk_device(seq["bgr"][sl], seq["disp"][sl], seq["flow"][sl],
                                          seq["mask"][sl])
        gb = ctx.bow_counters()
        gm = ctx.map_dump()
    finally:
        ctx.close()
    tr = oracle_mod.Tracker(W, H, (K["fx"], K["fy"], K["cx"], K["cy"]), bf, 0, nfeat)
    tr.set_vocabulary(VOC)
    ora = []
    for i in range(n):
        f = scene.to_numpy_frames({k: seq[k][i:i + 1] for k in ("bgr", "disp", "flow", "mask")})[0]
        ora.append(tr.track(f["bgr"], f["disp"], f["flow"], f["sem"]))
    return got, ora, gb, tr.bow_stats(), gm, tr.map_dump()


def _check_maps(gm, om):
    """Integer structure exact, poses / points / observations within 1e-3 (same_map; a key whose
    truncated pixel holds disparity 0 has depth bf / 0 = inf in the reference, Tracking.cc:447-456,
    and its point a non-finite position in both maps)."""
    from map_invariants import same_map
    diff, fmax = same_map(gm, om)
    assert diff == [] and fmax < 1e-3, (diff, fmax)
    assert np.abs(gm["kf_T"] - om["kf_T"]).max() < 1e-4


def test_vocabulary_tracking_three_quarter_res_matches_oracle(oracle_mod):
    """3/4-resolution C3 drive (the smallest the 8-level pyramid's cell grid takes), one
    textureless frame: the GPU tracker takes the oracle's
    TrackReferenceKeyFrame / Relocalization / CreateNewMapPoints path frame by frame (poses within
    the bar, integers exact), its vocabulary counters equal the oracle's, and the final map graph
    is the oracle's."""
    from multimot_track_amd import scene
    from oracle import compare
    K = {k: v * 0.75 for k, v in scene.KITTI03.items()}
    got, ora, gb, ob, gm, om = _run_pair(oracle_mod, 931, 281, K, K["bf"], 1000, 40, [24])
    rec = compare.parity_record(got, ora)
    assert rec["first_divergent_frame"] is None, rec
    assert {k: gb[k] for k in BOW_KEYS} == {k: ob[k] for k in BOW_KEYS}
    assert ob["trk_ok"] >= 1 and ob["reloc"] >= 1 and ob["triangulated"] > 0
    # frame 25 relocalises with 10-49 PoseOptimization inliers first: the SearchByProjection(F, KF,
    # sFound, 10, 100) round (Tracking.cc:3723-3753) runs on both sides, with equal outcomes
    assert ob["sbp_rounds"] >= 1 and ob["reloc_ok"] >= 1
    _check_maps(gm, om)


def test_vocabulary_tracking_c3_300_frames_matches_oracle(oracle_mod):
    """The C3 workload (1242x375, 2000 features, ego + 3 objects) over 300 frames with the
    vocabulary and two textureless frames: every frame matches the oracle, reference-keyframe
    tracking, relocalisation (with its SearchByProjection rounds) and triangulation all taken."""
    from multimot_track_amd import scene
    from oracle import compare
    K = dict(scene.KITTI03)
    got, ora, gb, ob, gm, om = _run_pair(oracle_mod, 1242, 375, K, 387.5744, 2000, 300,
                                         [120, 230], chunk=32)
    rec = compare.parity_record(got, ora)
    print("parity", rec, "\nbow counters", gb, "\nmap states", [g["map_state"] for g in got])
    assert rec["first_divergent_frame"] is None, rec
    assert {k: gb[k] for k in BOW_KEYS} == {k: ob[k] for k in BOW_KEYS}, (gb, ob)
    assert ob["trk_ok"] >= 1 and ob["reloc"] >= 2 and ob["triangulated"] > 100
    _check_maps(gm, om)


def _run_gpu(seq, n, chunk, W, H, K, bf, nfeat):
    import multimot_track_amd as M
    cfg = M.kitti03_config(W, H, nfeat, max_batch=chunk)
    cfg.fx, cfg.fy, cfg.cx, cfg.cy, cfg.bf = K["fx"], K["fy"], K["cx"], K["cy"], bf
    ctx = M.Context(cfg)
    got = []
    try:
        ctx.load_vocabulary(VOC)
        for s0 in range(0, n, chunk):
            sl = slice(s0, min(n, s0 + chunk))
            got += ctx.track_chunk_device(seq["bgr"][sl], seq["disp"][sl], seq["flow"][sl],
                                          seq["mask"][sl])
        return got, ctx.bow_counters(), ctx.map_dump()
    finally:
        ctx.close()


def _same(a, b):
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, np.ndarray):
        return a.shape == b.shape and np.array_equal(a, b, equal_nan=a.dtype.kind == "f")
    if isinstance(a, (float, np.floating)) and np.isnan(a):
        return isinstance(b, (float, np.floating)) and np.isnan(b)
    return a == b


def test_local_map_speculation_changes_nothing(monkeypatch, capfd):
    """UpdateLocalMap built from C2's matches while D1 runs (taken when D1's outliers leave the
    counted keyframe set unchanged, mmt_map.hip speculate_local_map / commit_local_map) and the
    object path beside the C3 chain: every frame's output, the vocabulary counters and the final
    map bit-identical to the build-as-you-go order (MMT_LOCALMAP_SPEC=0, MMT_OVERLAP_C3=0) over a
    C3 drive with a textureless frame (a relocalisation)."""
    import torch
    from multimot_track_amd import scene
    K = dict(scene.KITTI03)
    R = scene.SequenceRenderer(scene.StreetScene(3, 1003), 1242, 375, K=K,
                               device=torch.device("cuda:0"))
    n = 160
    seq = R.sequence(n)
    seq["bgr"][90] = 128
    args = (seq, n, 32, 1242, 375, K, 387.5744, 2000)
    monkeypatch.setenv("MMT_MAP_PROFILE", "1")  # the speculation counters, at destruction
    spec = _run_gpu(*args)
    import re
    m = re.search(r"speculated (\d+) times, taken (\d+)", capfd.readouterr().err)
    tries, hits = int(m.group(1)), int(m.group(2))
    print("local map speculated", tries, "taken", hits)
    assert tries > hits > 0  # both the taken and the discarded path ran
    monkeypatch.delenv("MMT_MAP_PROFILE")
    monkeypatch.setenv("MMT_LOCALMAP_SPEC", "0")
    monkeypatch.setenv("MMT_OVERLAP_C3", "0")
    base = _run_gpu(*args)
    assert spec[1]["reloc"] >= 1 and spec[1]["kfdb"] > 5
    assert _same(spec, base)
