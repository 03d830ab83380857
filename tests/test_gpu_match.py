"""GPU parity of the frame grid and projection matchers against the
CPU oracle through the C-ABI probes mmt_frame_grid / mmt_search_by_projection_frame /
mmt_search_local_points.  Integer and index outputs are bit-exact (the grid CSR, every binding of
a current key to a MapPoint, nmatches, isInFrustum's in-view flag and predicted level); the float
outputs (uR, depth, projections, view cosine) are bit-exact too."""
import numpy as np
import pytest

import match_problems as MP

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import multimot_track_amd as M
    c = M.Context(M.kitti03_config(nfeatures=2000))
    yield c
    c.close()


@pytest.mark.parametrize("fi", [0, 1, 3])
def test_frame_grid_bit_exact(ctx, oracle_mod, fi):
    k, _, dep = MP.frame(oracle_mod, fi)
    g = ctx.frame_grid(k, dep)
    o = oracle_mod.frame_stereo_grid(k, dep, MP.K, MP.BF)
    for a, b in zip(g, o):
        assert np.array_equal(a, b)


def test_frame_grid_edge_cases(ctx, oracle_mod):
    """No keys; keys on the image border (grid rounding to the last cells, out-of-grid keys);
    zero and infinite depth."""
    dep = np.zeros((MP.H, MP.W), np.float32)
    dep[:, ::2] = np.inf
    dep[::3, :] = 7.5
    empty = np.zeros(0, oracle_mod.KP_DTYPE)
    g = ctx.frame_grid(empty, dep)
    assert len(g[0]) == 0 and g[2][-1] == 0
    k = np.zeros(9, oracle_mod.KP_DTYPE)
    k["x"] = [0, 1241.9, 1241.0, 9.70, 9.71, 600, 19.40, 19.41, 0.5]
    k["y"] = [0, 374.9, 0, 3.9, 3.91, 187.5, 7.8, 7.82, 374.0]
    g = ctx.frame_grid(k, dep)
    o = oracle_mod.frame_stereo_grid(k, dep, MP.K, MP.BF)
    for a, b in zip(g, o):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("name", MP.SBP_CASES)
def test_search_by_projection_frame_matches_oracle(ctx, oracle_mod, name):
    c = MP.sbp_case(oracle_mod, name)
    args = (c["kps"], c["desc"], c["depth"], c["tcw"], c["last_kps"], c["Xw"], c["mp_desc"],
            c["active"], c["tlw"], c["th"])
    nm, match = ctx.search_by_projection_frame(*args, mono=c["mono"],
                                               check_orientation=c["check_orientation"],
                                               obs=c["obs"])
    onm, omatch = oracle_mod.search_by_projection_frame(*args, MP.K, MP.BF,
                                                        MP.scale_factors(oracle_mod),
                                                        c["mono"], c["check_orientation"],
                                                        obs=c["obs"])
    assert nm == onm
    assert np.array_equal(match, omatch), np.nonzero(match != omatch)[0][:10]


def test_search_by_projection_frame_empty(ctx, oracle_mod):
    c = MP.sbp_case(oracle_mod, "forward")
    nm, match = ctx.search_by_projection_frame(
        c["kps"], c["desc"], c["depth"], c["tcw"], c["last_kps"], c["Xw"], c["mp_desc"],
        np.zeros(len(c["last_kps"]), np.uint8), c["tlw"], 15.0)
    assert nm == 0 and np.all(match == -1)


@pytest.mark.parametrize("name", MP.LOCAL_CASES)
def test_search_local_points_matches_oracle(ctx, oracle_mod, name):
    c = MP.local_case(oracle_mod, name)
    args = (c["kps"], c["desc"], c["depth"], c["tcw"], c["Xw"], c["normal"], c["min_dist"],
            c["max_dist"], c["pdesc"], c["skip"], c["th"])
    nm, match, frus = ctx.search_local_points(*args, taken=c["taken"])
    onm, omatch, ofrus = oracle_mod.search_local_points(*args, MP.K, MP.BF,
                                                        MP.scale_factors(oracle_mod), c["taken"])
    assert np.array_equal(frus, ofrus)
    assert nm == onm
    assert np.array_equal(match, omatch), np.nonzero(match != omatch)[0][:10]
