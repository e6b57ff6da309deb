"""GPU parity: knnMatch(k=2) + ratio test vs the CPU restatement (bit-exact indices and distances).

Reference: /root/reference/src/TestsDetector.cpp:36,60 (BFMatcher NORM_L2 knnMatch k=2), :66-72.
"""
import numpy as np
import pytest

from computervision_objectdetection_featurematching_amd.synthetic import make_dataset, sift_like

pytestmark = pytest.mark.gpu


def _check(matcher, oracle, q, t):
    gi, gd = matcher.knn_match_arrays(q, t)
    oi, od = oracle.knn2(q, t)
    assert gi.shape == oi.shape
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gd.view(np.int32), od.view(np.int32))
    return gi, gd


@pytest.mark.parametrize("nq,nt", [(1, 1), (1, 2), (5, 3), (100, 1000), (333, 257), (2000, 2000), (700, 4100)])
def test_knn_sift_exact(matcher, oracle, nq, nt):
    rng = np.random.default_rng(nq * 7919 + nt)
    _check(matcher, oracle, sift_like(rng, nq), sift_like(rng, nt))


def test_knn_planted_dataset(matcher, oracle):
    ds = make_dataset(1, 1, 2000, 2000, 400)
    gi, gd = _check(matcher, oracle, ds.model_desc[0], ds.scene_desc[0])
    # planted rows find their copies
    assert (gi[:400, 0] == ds.plant_pos[0, 0]).mean() > 0.99


def test_knn_ties_lower_index(matcher, oracle):
    rng = np.random.default_rng(5)
    t = sift_like(rng, 300)
    t[200] = t[17]          # exact duplicate train rows -> tie, lower index first
    t[250] = t[17]
    q = np.stack([t[17], t[42], t[250]])
    gi, gd = _check(matcher, oracle, q, t)
    assert gi[0, 0] == 17 and gi[0, 1] == 200 and gd[0, 0] == 0 and gd[0, 1] == 0


def test_knn_large_values_sqrt_collisions(matcher, oracle):
    # 0/255 patterns give squared distances up to 128*255^2 where distinct integers share a float sqrt
    rng = np.random.default_rng(11)
    q = (rng.integers(0, 2, size=(64, 128)) * 255).astype(np.float32)
    t = (rng.integers(0, 2, size=(1500, 128)) * 255).astype(np.float32)
    t[::7] = np.clip(t[::7] + rng.integers(-3, 4, size=t[::7].shape), 0, 255)
    _check(matcher, oracle, q, t)


def test_knn_generic_float(matcher, oracle):
    rng = np.random.default_rng(3)
    q = rng.normal(size=(300, 128)).astype(np.float32)
    t = rng.normal(size=(900, 128)).astype(np.float32)
    _check(matcher, oracle, q, t)


def test_knn_empty_train_and_query(matcher, oracle):
    rng = np.random.default_rng(1)
    q = sift_like(rng, 10)
    gi, gd = matcher.knn_match_arrays(q, np.zeros((0, 128), np.float32))
    assert (gi == -1).all()
    gi, gd = matcher.knn_match_arrays(np.zeros((0, 128), np.float32), q)
    assert gi.shape == (0, 2)
    assert matcher.knn_match(np.zeros((0, 128), np.float32), q) == []


def test_ratio_filter(matcher, oracle):
    ds = make_dataset(1, 1, 1000, 1500, 300)
    oi, od = oracle.knn2(ds.model_desc[0], ds.scene_desc[0])
    gq, gt = matcher.ratio_filter(oi, od, 0.9)
    rq, rt = oracle.ratio_filter(oi, od, 0.9)
    np.testing.assert_array_equal(gq, rq)
    np.testing.assert_array_equal(gt, rt)
    # boundary: d0 == 0.9f*d1 exactly is rejected (strict <)
    idx = np.array([[1, 2], [3, -1], [4, 5]], np.int32)
    d1 = np.float32(10.0)
    dist = np.array([[np.float32(0.9) * d1, d1], [1, 0], [np.nextafter(np.float32(0.9) * d1, 0), d1]], np.float32)
    gq, gt = matcher.ratio_filter(idx, dist, 0.9)
    np.testing.assert_array_equal(gq, [2])
    np.testing.assert_array_equal(gt, [4])


def test_knn_late_tile_ties_across_row_halves(matcher, oracle):
    # the late-tile filter keeps a row iff D <= the lane pair's 2nd best; duplicates of the query's
    # nearest rows placed late, in both row halves of a 32-row block (rows 4h..4h+3 of every 8) and
    # across tiles, must come out in index order
    rng = np.random.default_rng(23)
    t = sift_like(rng, 3000)
    q = sift_like(rng, 40)
    for j in range(40):
        pos = np.sort(rng.choice(np.arange(300, 3000), size=5, replace=False))
        pos[1] = pos[0] + 4 if pos[0] + 4 < pos[2] else pos[1]  # other half of the same 8-row group
        for p in pos:
            t[p] = q[j]
    _check(matcher, oracle, q, t)


def test_knn_small_pool_mass_ties(matcher, oracle):
    # 4,096 train rows drawn from 24 distinct descriptors: every query's best and 2nd best are tied
    # many times over, in every tile and both row halves
    rng = np.random.default_rng(29)
    pool = sift_like(rng, 24)
    t = pool[rng.integers(0, 24, size=4096)]
    q = np.concatenate([pool[rng.integers(0, 24, size=100)], sift_like(rng, 100)])
    gi, _ = _check(matcher, oracle, q, t)
    assert (gi[:100, 0] < gi[:100, 1]).all()  # equal distance: lower index first


def test_knn_split_tail_identical(oracle):
    """MIM_KNN_TAIL=1 (opt-in): when the query-block sweeps leave the last round of resident blocks partly
    empty, the trailing problems run as train-tile pieces whose partial top-2 lists the ratio kernel
    merges.  40 problems x 16 sweeps = 640 sweeps over 512 resident blocks: the records and good-match
    lists equal the whole-sweep schedule's, and a sampled problem equals the oracle."""
    import os

    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(1, 40, 8000, 2500, 600, inlier_frac=0.3, seed=77)
    outs = []
    for tail in ("0", "1"):
        os.environ["MIM_KNN_TAIL"] = tail
        m = Matcher(0)
        try:
            q = m.add_set(ds.model_desc[0], ds.model_kp[0])
            ts = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q, t) for t in ts], default_params(max_iters=500))
            det = [m.problem_detail(i, int(r["n_good"])) for i, r in enumerate(res)]
        finally:
            m.close()
            os.environ.pop("MIM_KNN_TAIL", None)
        outs.append((res, det))
    (r0, d0), (r1, d1) = outs
    assert r0.tobytes() == r1.tobytes()
    for a, b in zip(d0, d1):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    o = oracle.match_problem(ds.model_desc[0], ds.model_kp[0], ds.scene_desc[39], ds.scene_kp[39],
                             oracle.default_params(max_iters=500))
    assert int(r1[39]["n_good"]) == o["n_good"] and np.array_equal(d1[39][0], o["good_q"])
