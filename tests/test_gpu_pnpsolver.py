"""Row D6 on the GPU: PnPsolver (ORB-SLAM2's P4P EPnP-RANSAC of Tracking::Relocalization)
through mmt_pnpsolver_iterate, against the CPU oracle (oracle/pnp_ref.cpp) on the same inputs
and the same RandomInt draws (glibc rand() stream, restatement pinned in
tests/test_oracle_pnpsolver.py).

Tolerance: iterations, found / no_more, inlier counts and masks, the solver state exact; poses
within 1e-4 (the 4-point hypotheses' EPnP is operation for operation the checker's; Refine()'s
sums over the inliers are reduced in a different order).  The camera intrinsics are float, as
Frame's fx..cy that PnPsolver copies into its doubles."""
import numpy as np
import pytest

from synth_problems import K_KITTI, p4p_problem

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4
PARAMS = (0.99, 10, 300, 4, 0.5, 5.991)


@pytest.fixture(scope="module")
def ctx():
    import multimot_track_amd as M
    c = M.Context(M.kitti03_config(nfeatures=2000))
    yield c
    c.close()


def _compare(g, o, gs, os_):
    assert g["found"] == o["found"] and g["no_more"] == o["no_more"]
    assert g["n_inliers"] == o["n_inliers"]
    assert np.array_equal(g["mask"], o["mask"])
    assert gs["iterations"] == os_["iterations"] and gs["best_inliers"] == os_["best_inliers"]
    assert np.array_equal(gs["best_mask"], os_["best_mask"])
    if g["found"]:  # refined pose, or mBestTcw once the iterations are exhausted
        assert np.abs(g["Tcw"] - o["Tcw"]).max() < POSE_TOL
    if gs["best_inliers"]:
        assert np.abs(gs["best_Tcw"] - os_["best_Tcw"]).max() < POSE_TOL


@pytest.mark.parametrize("seed,n,out,noise", [(0, 120, 0.0, 0.0), (1, 200, 0.3, 0.3),
                                              (2, 400, 0.45, 0.5), (3, 60, 0.2, 1.0),
                                              (4, 1500, 0.5, 0.5), (6, 15, 0.0, 0.5)])
def test_pnpsolver_matches_oracle(ctx, oracle_mod, seed, n, out, noise):
    p3, p2, s2, _ = p4p_problem(seed, n, outlier_frac=out, pix_noise=noise)
    randi = oracle_mod.p4p_randi(n, 400, seed + 1)
    gs, os_ = {}, {}
    g = ctx.pnpsolver_iterate(p3, p2, s2, K_KITTI, randi, 5, gs, PARAMS)
    o = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, randi, 5, os_, PARAMS)
    _compare(g, o, gs, os_)


def test_pnpsolver_state_carries_across_calls(ctx, oracle_mod):
    """Relocalization calls iterate(5) again on the same solver when the returned pose is
    rejected later (Tracking.cc:3672-3760): the second call continues the iteration count and
    the best set; its draws continue the rand() stream."""
    n = 300
    p3, p2, s2, _ = p4p_problem(7, n, outlier_frac=0.35, pix_noise=0.5)
    draws = oracle_mod.p4p_randi(n, 800, 7)
    gs, os_ = {}, {}
    g = ctx.pnpsolver_iterate(p3, p2, s2, K_KITTI, draws[:400], 5, gs, PARAMS)
    o = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, draws[:400], 5, os_, PARAMS)
    _compare(g, o, gs, os_)
    used = gs["iterations"]
    g = ctx.pnpsolver_iterate(p3, p2, s2, K_KITTI, draws[used:], 5, gs, PARAMS)
    o = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, draws[used:], 5, os_, PARAMS)
    _compare(g, o, gs, os_)
    assert gs["iterations"] > used


def test_pnpsolver_all_outliers_and_too_few(ctx, oracle_mod):
    n = 60
    p3, p2, s2, _ = p4p_problem(5, n, outlier_frac=0.0)
    rng = np.random.default_rng(5)
    p2 = np.stack([rng.uniform(0, 1242, n), rng.uniform(0, 375, n)], 1).astype(np.float32)
    randi = oracle_mod.p4p_randi(n, 400, 3)
    gs, os_ = {}, {}
    g = ctx.pnpsolver_iterate(p3, p2, s2, K_KITTI, randi, 5, gs, PARAMS)
    o = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, randi, 5, os_, PARAMS)
    _compare(g, o, gs, os_)
    assert g["no_more"] and not g["found"] and gs["iterations"] == 35
    g = ctx.pnpsolver_iterate(p3[:9], p2[:9], s2[:9], K_KITTI, randi, 5, {}, PARAMS)
    assert g["no_more"] and not g["found"]


def test_pnpsolver_rejects_bad_arguments(ctx):
    import multimot_track_amd as M
    p3, p2, s2, _ = p4p_problem(8, 50, outlier_frac=0.0)
    with pytest.raises(M.MmtError):
        ctx.pnpsolver_iterate(p3, p2, s2, K_KITTI, np.zeros((2, 4), np.int32), 5, {}, PARAMS)
    with pytest.raises(M.MmtError):
        ctx.pnpsolver_iterate(p3, p2, s2, K_KITTI, np.zeros((400, 4), np.int32), 5, {},
                              (0.99, 10, 300, 5, 0.5, 5.991))
