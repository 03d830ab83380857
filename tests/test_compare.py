"""CPU tests of the parity bar itself (oracle/compare.py): integer outputs exact, poses within
1e-4 or 4 float32 ulps, centroids within 1e-3, LM iteration counts reported as stop flips when
the solve's pose is within the bar."""
import numpy as np

from oracle import compare


def frame(pose_shift=0.0, iters=7, obj_iters=12, inliers=300, X_shift=0.0):
    T = np.eye(4, dtype=np.float32)
    T[0, 3] = 1.0 + pose_shift
    X = np.eye(4, dtype=np.float32)
    X[2, 3] = 0.5 + X_shift
    ob = dict(label=1, sem_label=2, n_points=900, ransac_inliers=400, mm_inliers=-1, n_solve=400,
              n_inliers=inliers, iterations=obj_iters, init=X.copy(), X=X, motion=X.copy(),
              centre_pre=np.array([1.0, 2.0, 3.0], np.float32))
    return dict(initialized=1, n_keys=2000, n_obj_samples=5000, ego_iterations=iters,
                ego_inliers=1500, Tcw=T, objects=[ob])


def test_identical_frames_pass():
    rec = compare.parity_record([frame()], [frame()])
    assert rec["first_divergent_frame"] is None and rec["lm_stop_flips"] == 0


def test_integer_mismatch_diverges():
    rec = compare.parity_record([frame(inliers=301)], [frame()])
    assert rec["first_divergent_frame"] == 0 and "n_inliers" in rec["first_divergence"]


def test_pose_outside_the_bar_diverges():
    rec = compare.parity_record([frame(pose_shift=3e-4)], [frame()])
    assert rec["first_divergent_frame"] == 0


def test_lm_iteration_mismatch_with_pose_in_bar_is_a_stop_flip():
    rec = compare.parity_record([frame(), frame(obj_iters=28, X_shift=2e-6)],
                                [frame(), frame(obj_iters=5)])
    assert rec["first_divergent_frame"] is None
    assert rec["lm_stop_flips"] == 1 and rec["first_lm_stop_flip"] == 1


def test_lm_iteration_mismatch_with_pose_outside_the_bar_diverges():
    rec = compare.parity_record([frame(obj_iters=28, X_shift=5e-3)], [frame(obj_iters=5)])
    assert rec["first_divergent_frame"] == 0 and rec["lm_stop_flips"] == 1
