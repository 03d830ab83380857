"""GPU parity of SearchByBoW against the CPU oracle through the C-ABI probe
mmt_search_by_bow: every binding and nmatches bit-exact, for the reference's two ratios (0.7
TrackReferenceKeyFrame, 0.75 Relocalization), with and without the rotation check, in-node list
orders shuffled, nodes larger than a wave (up to the 2048-feature node limit), invalid MapPoints,
and the argument checks (a feature listed in two nodes, node ids out of order)."""
import numpy as np
import pytest

import bow_problems as BP

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import multimot_track_amd as M
    c = M.Context(M.kitti03_config(nfeatures=2000))
    yield c
    c.close()


@pytest.mark.parametrize("seed,kw,ratio,orient", [
    (0, {}, 0.7, True),
    (1, {"shuffle": True}, 0.75, True),
    (2, {"n_nodes": 10}, 0.7, True),              # ~200 frame features per node (4 chunks)
    (3, {"n_nodes": 1, "n_f": 2000}, 0.7, True),  # one node of 2000 features (32 chunks)
    (4, {"n_kf": 4000, "n_f": 8000, "n_nodes": 900}, 0.7, True),
    (5, {"mp_valid": 0.3}, 0.7, False),
    (6, {"frac_match": 0.0}, 0.7, True),
    (7, {"rot_outliers": 0.6, "dup": 0.3}, 0.75, True),
])
def test_search_by_bow_matches_oracle(ctx, oracle_mod, seed, kw, ratio, orient):
    pr = BP.bow_problem(seed, **kw)
    nm_o, m_o = oracle_mod.search_by_bow(*pr, nnratio=ratio, check_orientation=orient)
    nm_g, m_g = ctx.search_by_bow(*pr, nnratio=ratio, check_orientation=orient)
    assert nm_g == nm_o
    assert np.array_equal(m_g, m_o), np.nonzero(m_g != m_o)[0][:10]
    if kw.get("frac_match", 0.6) > 0:
        assert nm_o > 20


def test_search_by_bow_empty(ctx, oracle_mod):
    pr = BP.bow_problem(11, n_kf=50, n_f=60)
    empty = (np.zeros(0, np.uint32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    nm, m = ctx.search_by_bow(empty, pr[1], pr[2], pr[3], pr[4], pr[5], pr[6])
    assert nm == 0 and (m == -1).all()
    nm, m = ctx.search_by_bow(pr[0], pr[1], pr[2], pr[3], empty, pr[5], pr[6])
    assert nm == 0 and (m == -1).all()


def test_search_by_bow_rejects_bad_vectors(ctx):
    import multimot_track_amd as M
    pr = BP.bow_problem(12, n_kf=50, n_f=60)
    node, start, feat = pr[4]
    twice = (node, start, np.concatenate([feat[:-1], feat[:1]]))
    with pytest.raises(M.MmtError):
        ctx.search_by_bow(pr[0], pr[1], pr[2], pr[3], twice, pr[5], pr[6])
    unsorted = (node[::-1].copy(), start, feat)
    with pytest.raises(M.MmtError):
        ctx.search_by_bow(pr[0], pr[1], pr[2], pr[3], unsorted, pr[5], pr[6])
