"""Row D6 (PnPsolver, ORB-SLAM2's P4P EPnP-RANSAC of Tracking::Relocalization) -- CPU checker.

The oracle restates PnPsolver.cc:67-339 (SetRansacParameters, iterate, Refine, CheckInliers) on
top of the EPnP restatement, and glibc's rand() (the stream DUtils::Random::RandomInt draws
from, Thirdparty/DBoW2/DUtils/Random.cpp:47-50).  The rand() restatement is pinned against this
container's libc; the solver against exact geometry and the reference's control flow."""
import ctypes
import ctypes.util

import numpy as np
import pytest

from synth_problems import K_KITTI, p4p_problem

PARAMS = (0.99, 10, 300, 4, 0.5, 5.991)  # Tracking.cc:3659 SetRansacParameters


@pytest.mark.parametrize("seed", [1, 42, 12345, 0])
def test_glibc_rand_restatement_matches_libc(oracle_mod, seed):
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.srand(ctypes.c_uint(seed))
    ref = np.array([libc.rand() for _ in range(2000)], np.int64)
    got = oracle_mod.glibc_rand(seed, 2000).astype(np.int64)
    assert np.array_equal(got, ref)


def test_p4p_draws_stay_in_range(oracle_mod):
    r = oracle_mod.p4p_randi(37, 500, 1)
    for j in range(4):
        assert r[:, j].min() >= 0 and r[:, j].max() <= 36 - j


def _rel_pose_err(T, Tt):
    return float(np.abs(T.astype(np.float64) - Tt).max())


def test_exact_geometry_found_at_first_iteration(oracle_mod):
    p3, p2, s2, T = p4p_problem(0, 120, outlier_frac=0.0, pix_noise=0.0)
    st = {}
    r = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, oracle_mod.p4p_randi(120, 400), 5, st,
                                     PARAMS)
    assert r["found"] and not r["no_more"]
    assert st["iterations"] == 1 and r["n_inliers"] == 120 and r["mask"].all()
    assert _rel_pose_err(r["Tcw"], T) < 1e-4


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_outliers_rejected(oracle_mod, seed):
    n = 200
    p3, p2, s2, T = p4p_problem(seed, n, outlier_frac=0.3, pix_noise=0.3)
    r = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, oracle_mod.p4p_randi(n, 400), 5, {},
                                     PARAMS)
    assert r["found"]
    assert _rel_pose_err(r["Tcw"], T) < 0.05
    assert r["n_inliers"] >= 0.55 * n


def test_too_few_correspondences(oracle_mod):
    p3, p2, s2, _ = p4p_problem(4, 9, outlier_frac=0.0)
    r = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, oracle_mod.p4p_randi(9, 10), 5, {},
                                     PARAMS)
    assert r["no_more"] and not r["found"]


def test_all_outliers_exhaust_iterations(oracle_mod):
    n = 60
    p3, p2, s2, _ = p4p_problem(5, n, outlier_frac=0.0)
    rng = np.random.default_rng(5)
    p2 = np.stack([rng.uniform(0, 1242, n), rng.uniform(0, 375, n)], 1).astype(np.float32)
    st = {}
    r = oracle_mod.pnpsolver_iterate(p3, p2, s2, K_KITTI, oracle_mod.p4p_randi(n, 400), 5, st,
                                     PARAMS)
    assert r["no_more"] and not r["found"]
    # SetRansacParameters: minInliers = max(10, n*0.5) = 30, eps = 0.5 -> 35 iterations
    assert st["iterations"] == 35
