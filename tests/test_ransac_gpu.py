"""GPU parity: findHomography(RANSAC) and the fused per-problem path vs the CPU restatement.

Reference: /root/reference/src/TestsDetector.cpp:74-94 (gates, findHomography(objPts, scenePts,
RANSAC, 5.0, inlierMask), countNonZero, determinant, inlier gather).
Contract: inlier masks identical, RANSAC iteration counts identical, H within 1e-4
(tested tighter: the minimal-sample arithmetic is bit-exact; only the refit/LM summation order
differs between the CPU restatement and the device block reductions).
"""
import numpy as np
import pytest

from computervision_objectdetection_featurematching_amd.synthetic import apply_h, make_dataset, random_homography

pytestmark = pytest.mark.gpu
H_RTOL = 0.0  # bit-identical H (refit + LM in the oracle's operation order)


def _points(n, w, seed, noise=0.5):
    rng = np.random.default_rng(seed)
    H = random_homography(rng)
    src = np.c_[rng.uniform(0, 640, n), rng.uniform(0, 480, n)].astype(np.float32)
    dst = np.c_[rng.uniform(0, 640, n), rng.uniform(0, 480, n)].astype(np.float32)
    k = int(round(w * n))
    inl = rng.choice(n, size=k, replace=False)
    dst[inl] = apply_h(H, src[inl]) + rng.uniform(-noise, noise, size=(k, 2)).astype(np.float32)
    return src, dst, H


def _cmp_h(Hg, Ho):
    assert np.max(np.abs(Hg - Ho) / (np.abs(Ho) + 1e-3)) <= H_RTOL, (Hg, Ho)


@pytest.mark.parametrize("n,w,iters", [(5, 1.0, 2000), (6, 0.5, 2000), (7, 0.3, 3000), (9, 0.5, 2000), (12, 0.8, 2000), (60, 0.5, 2000), (200, 0.3, 2000),
                                       (500, 0.15, 2000), (1000, 0.08, 5000), (3000, 0.25, 2000)])
def test_find_homography_matches_oracle(matcher, oracle, n, w, iters):
    src, dst, _ = _points(n, w, seed=n * 31 + iters)
    Hg, mg = matcher.find_homography(src, dst, 5.0, iters, 0.995)
    ok, Ho, mo = oracle.find_homography(src, dst, 5.0, iters, 0.995)
    assert (Hg is not None) == bool(ok)
    np.testing.assert_array_equal(mg, mo)
    if ok:
        _cmp_h(Hg, Ho)


def test_find_homography_ransac_trace(matcher, oracle):
    # iteration count / best iteration of the restated loop are reproduced through the batch path
    src, dst, _ = _points(400, 0.3, seed=7)
    r = oracle.ransac(src, dst, 5.0, 0.995, 2000)
    Hg, mg = matcher.find_homography(src, dst, 5.0, 2000, 0.995)
    np.testing.assert_array_equal(mg, r["mask"])


def test_exact_recovery_noiseless(matcher):
    rng = np.random.default_rng(2)
    H = random_homography(rng)
    src = np.c_[rng.uniform(0, 640, 50), rng.uniform(0, 480, 50)].astype(np.float32)
    dst = apply_h(H, src)
    Hg, mg = matcher.find_homography(src, dst)
    assert mg.all()
    np.testing.assert_allclose(Hg, H / H[2, 2], rtol=1e-4, atol=1e-6)


def test_four_points_direct(matcher, oracle):
    src = np.array([[0, 0], [100, 0], [100, 80], [0, 80]], np.float32)
    dst = np.array([[10, 5], [120, 8], [115, 95], [7, 90]], np.float32)
    Hg, mg = matcher.find_homography(src, dst)
    ok, Ho, mo = oracle.find_homography(src, dst)
    assert ok and Hg is not None
    np.testing.assert_array_equal(mg, [1, 1, 1, 1])
    np.testing.assert_array_equal(mg, mo)
    assert np.array_equal(Hg, Ho)  # n == 4: runKernel only, bit-exact


def test_degenerate_returns_empty(matcher, oracle):
    src = np.tile(np.array([[5.0, 7.0]], np.float32), (10, 1))
    dst = np.tile(np.array([[1.0, 2.0]], np.float32), (10, 1))
    Hg, mg = matcher.find_homography(src, dst)
    ok, Ho, mo = oracle.find_homography(src, dst)
    assert not ok and Hg is None
    assert not mg.any()


def test_too_few_points_raises(matcher):
    with pytest.raises(ValueError):
        matcher.find_homography(np.zeros((3, 2), np.float32), np.zeros((3, 2), np.float32))


def _batch_vs_oracle(matcher, oracle, ds, max_iters):
    matcher.clear_sets()
    q_ids = [matcher.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
    t_ids = [matcher.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
    probs = [(q_ids[m], t_ids[s]) for m, s in ds.problems]
    from computervision_objectdetection_featurematching_amd import default_params
    prm = default_params(max_iters=max_iters)
    res = matcher.match_batch(probs, prm)
    oprm = oracle.default_params(max_iters=max_iters)
    for i, (m, s) in enumerate(ds.problems):
        o = oracle.match_problem(ds.model_desc[m], ds.model_kp[m], ds.scene_desc[s], ds.scene_kp[s], oprm)
        r = res[i]
        assert r["n_good"] == o["n_good"], i
        gq, gt, gm = matcher.problem_detail(i, int(r["n_good"]))
        np.testing.assert_array_equal(gq, o["good_q"])
        np.testing.assert_array_equal(gt, o["good_t"])
        assert r["status"] == o["status"], (i, r["status"], o["status"])
        assert r["n_inl"] == o["n_inl"], i
        if o["n_good"] > 4:
            assert r["iters"] == o["iters"], i
            np.testing.assert_array_equal(gm, o["mask"])
        if o["status"] != 2 and o["n_good"] >= 4:
            _cmp_h(r["H"].reshape(3, 3), o["H"])
    return res


def test_batch_c2_shape(matcher, oracle):
    ds = make_dataset(1, 1, 2000, 2000, 400)
    _batch_vs_oracle(matcher, oracle, ds, 2000)


def test_batch_multi_problem_high_inlier(matcher, oracle):
    # high inlier fraction: adaptive termination (niters) kicks in early
    ds = make_dataset(2, 3, 600, 1500, 200, inlier_frac=0.6, seed=77)
    res = _batch_vs_oracle(matcher, oracle, ds, 2000)
    assert (res["iters"] < 2000).all()


def test_batch_ragged_and_gates(matcher, oracle):
    # mixes problems with < 4 good matches, exactly 4, and regular ones
    ds = make_dataset(2, 2, 300, 900, 100, inlier_frac=0.3, seed=9)
    ds.model_desc.append(ds.model_desc[0][:3].copy())
    ds.model_kp.append(ds.model_kp[0][:3].copy())
    ds.model_desc.append(ds.model_desc[1][:4].copy())
    ds.model_kp.append(ds.model_kp[1][:4].copy())
    _batch_vs_oracle(matcher, oracle, ds, 1000)


def _adversarial_sets():
    rng = np.random.default_rng(99)
    out = []
    # clustered + near-collinear points (stress the conditioning screen of the filtered path)
    n = 300
    t = rng.uniform(0, 1, n)
    src = np.c_[100 + 400 * t, 200 + 1e-3 * rng.normal(size=n)].astype(np.float32)
    src[::3] = np.c_[rng.uniform(0, 640, len(src[::3])), rng.uniform(0, 480, len(src[::3]))]
    H = random_homography(rng)
    dst = apply_h(H, src) + rng.normal(scale=0.7, size=src.shape).astype(np.float32)
    dst[::4] = np.c_[rng.uniform(0, 640, len(dst[::4])), rng.uniform(0, 480, len(dst[::4]))]
    out.append((src, dst))
    # duplicated points
    src2 = np.repeat(np.c_[rng.uniform(0, 640, 40), rng.uniform(0, 480, 40)], 5, axis=0).astype(np.float32)
    dst2 = apply_h(random_homography(rng), src2)
    dst2[::3] += rng.normal(scale=30, size=dst2[::3].shape).astype(np.float32)
    out.append((src2, dst2))
    # large coordinates (4k scenes) and strong perspective
    src3 = np.c_[rng.uniform(0, 4096, 500), rng.uniform(0, 3000, 500)].astype(np.float32)
    H3 = random_homography(rng)
    H3[2, :2] = [2e-4, -1.5e-4]
    dst3 = apply_h(H3, src3) + rng.normal(scale=1.0, size=src3.shape).astype(np.float32)
    dst3[::2] = np.c_[rng.uniform(0, 4096, 250), rng.uniform(0, 3000, 250)]
    out.append((src3, dst3))
    # points exactly on the threshold ring: err == 25 ties
    src4 = np.c_[rng.uniform(0, 640, 200), rng.uniform(0, 480, 200)].astype(np.float32)
    dst4 = src4 + np.float32(5.0) * np.c_[np.cos(np.arange(200)), np.sin(np.arange(200))].astype(np.float32)
    dst4[:60] = src4[:60]
    out.append((src4, dst4))
    return out


@pytest.mark.parametrize("case", range(4))
def test_find_homography_adversarial(matcher, oracle, case):
    src, dst = _adversarial_sets()[case]
    for iters in (2000, 20000):
        Hg, mg = matcher.find_homography(src, dst, 5.0, iters, 0.995)
        ok, Ho, mo = oracle.find_homography(src, dst, 5.0, iters, 0.995)
        assert (Hg is not None) == bool(ok)
        np.testing.assert_array_equal(mg, mo)
        if ok:
            assert np.max(np.abs(Hg - Ho) / (np.abs(Ho) + 1e-3)) < 1e-6


def test_filtered_equals_exact_all(oracle):
    """The default filtered RANSAC and the all-hypotheses-exact reference mode give identical output."""
    import os
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(3, 4, 1500, 2500, 500, inlier_frac=0.08, seed=31337)
    outs = []
    for mode in ("0", "1"):
        os.environ["MIM_RANSAC_EXACT"] = mode
        m = Matcher(0)
        try:
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=20000))
            masks = [m.problem_detail(i, int(r["n_good"]))[2] for i, r in enumerate(res)]
            sets = _adversarial_sets()
            fh = [m.find_homography(s, d, 5.0, 5000) for s, d in sets]
        finally:
            m.close()
            os.environ.pop("MIM_RANSAC_EXACT", None)
        outs.append((res, masks, fh))
    (r0, m0, f0), (r1, m1, f1) = outs
    assert r0.tobytes() == r1.tobytes()
    for a, b in zip(m0, m1):
        np.testing.assert_array_equal(a, b)
    for (ha, ma), (hb, mb) in zip(f0, f1):
        np.testing.assert_array_equal(ma, mb)
        assert (ha is None) == (hb is None) and (ha is None or np.array_equal(ha, hb))


def test_bound_mfma_equals_exact_all():
    """RANSAC bounds the inlier counts on the matrix cores (f16 hi/lo split GEMMs) and evaluates only
    the candidates exactly; the all-exact reference mode (MIM_RANSAC_EXACT=1: runKernel + computeError
    for every iteration) must give the identical output (the bounds are only filters)."""
    import os
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(2, 3, 1500, 2500, 500, inlier_frac=0.08, seed=2718)
    sets = _adversarial_sets()
    outs = []
    for key, mode in (("MIM_RANSAC_EXACT", "0"), ("MIM_RANSAC_EXACT", "1")):
        os.environ[key] = mode
        m = Matcher(0)
        try:
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=12000))
            masks = [m.problem_detail(i, int(r["n_good"]))[2] for i, r in enumerate(res)]
            fh = []
            for s_, d_ in sets:
                fh.append(m.find_homography(s_, d_, 5.0, 12000) + (m.batch_results(1).tobytes(),))
        finally:
            m.close()
            os.environ.pop(key, None)
        outs.append((res, masks, fh))
    r0, m0, f0 = outs[0]
    for r1, m1, f1 in outs[1:]:
        assert r0.tobytes() == r1.tobytes()
        for a, b in zip(m0, m1):
            np.testing.assert_array_equal(a, b)
        for (ha, ma, ra), (hb, mb, rb) in zip(f0, f1):
            np.testing.assert_array_equal(ma, mb)
            assert ra == rb


def test_mostly_degenerate_points(matcher, oracle):
    """Most 4-subsets collinear: long runs of rejected getSubset attempts, many redraws."""
    rng = np.random.default_rng(17)
    src = np.c_[np.arange(40, dtype=np.float32) * 7, np.full(40, 100, np.float32)]   # all on one line
    src[-3:] = rng.uniform(0, 400, size=(3, 2))                                          # 3 off-line points
    dst = src * np.float32(1.1) + np.float32(3)
    for iters in (50, 2000):
        Hg, mg = matcher.find_homography(src, dst, 5.0, iters, 0.995)
        ok, Ho, mo = oracle.find_homography(src, dst, 5.0, iters, 0.995)
        assert (Hg is not None) == bool(ok)
        np.testing.assert_array_equal(mg, mo)


@pytest.mark.parametrize("groups", ["2", "3"])
def test_grouped_pipeline_identical(groups):
    """Pipelined groups (problem ranges on their own streams) give the same records as one stream."""
    import os
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(2, 5, 1200, 2000, 400, inlier_frac=0.1, seed=4242)
    outs = []
    for g in ("1", groups):
        os.environ["MIM_GROUPS"] = g
        m = Matcher(0)
        try:
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=8000))
            masks = [m.problem_detail(i, int(r["n_good"]))[2] for i, r in enumerate(res)]
        finally:
            m.close()
            os.environ.pop("MIM_GROUPS", None)
        outs.append((res, masks))
    (r0, m0), (r1, m1) = outs
    assert r0.tobytes() == r1.tobytes()
    for a, b in zip(m0, m1):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("n_off,iters", [(0, 2000), (3, 2000), (4, 20000)])
def test_chain_sampler_rejection_runs(matcher, oracle, n_off, iters):
    """n large enough for the chain sampler (few repeated-index redraws) with most subsets collinear:
    runs of rejected attempts up to and past getSubset's 10000-attempt limit.  The refit of such a
    degenerate inlier set is ill-conditioned, so the check is on the RANSAC trace, not on H."""
    rng = np.random.default_rng(100 + n_off)
    n = 300
    src = np.c_[np.arange(n, dtype=np.float32) * 2, np.full(n, 100, np.float32)]
    if n_off:
        src[-n_off:] = rng.uniform(0, 400, size=(n_off, 2)).astype(np.float32)
    dst = src * np.float32(1.1) + np.float32(3)
    Hg, mg = matcher.find_homography(src, dst, 5.0, iters, 0.995)
    rec = matcher.batch_results(1)[0]
    r = oracle.ransac(src, dst, 5.0, 0.995, iters)
    assert (Hg is not None) == bool(r["ok"])
    np.testing.assert_array_equal(mg, r["mask"])
    assert rec["iters"] == r["iters"], (rec["iters"], r["iters"])


def test_chain_sampler_equals_walker():
    """The chain sampler and the attempt-by-attempt walker (MIM_SAMPLER_WALK=1) give identical output."""
    import os
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(2, 3, 1500, 2500, 500, inlier_frac=0.08, seed=777)
    sets = _adversarial_sets()
    outs = []
    for mode in ("0", "1"):
        os.environ["MIM_SAMPLER_WALK"] = mode
        m = Matcher(0)
        try:
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=30000))
            masks = [m.problem_detail(i, int(r["n_good"]))[2] for i, r in enumerate(res)]
            fh = []
            for s_, d_ in sets:
                fh.append(m.find_homography(s_, d_, 5.0, 20000) + (m.batch_results(1).tobytes(),))
        finally:
            m.close()
            os.environ.pop("MIM_SAMPLER_WALK", None)
        outs.append((res, masks, fh))
    (r0, m0, f0), (r1, m1, f1) = outs
    assert r0.tobytes() == r1.tobytes()
    for a, b in zip(m0, m1):
        np.testing.assert_array_equal(a, b)
    for (ha, ma, ra), (hb, mb, rb) in zip(f0, f1):
        np.testing.assert_array_equal(ma, mb)
        assert ra == rb


def test_concurrent_contexts_identical():
    """Two contexts with batches in flight at once on their own streams (bench.py --inflight 2) give
    the records and masks of one context run alone: contexts share no device state."""
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(2, 4, 1200, 2000, 400, inlier_frac=0.1, seed=777)
    prm = default_params(max_iters=8000)
    pairs = ds.problems

    def run(ms):
        for m in ms:  # enqueue every context's batch before collecting any
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            m.match_batch_async([(q[a], t[b]) for a, b in pairs], prm)
        out = []
        for m in ms:
            res = m.batch_results(len(pairs))
            out.append((res, [m.problem_detail(i, int(r["n_good"]))[2] for i, r in enumerate(res)]))
        return out

    solo = Matcher(0)
    duo = [Matcher(0), Matcher(0)]
    try:
        (r0, m0), = run([solo])
        for r1, m1 in run(duo):
            assert r0.tobytes() == r1.tobytes()
            for a, b in zip(m0, m1):
                np.testing.assert_array_equal(a, b)
    finally:
        for m in [solo] + duo:
            m.close()


def test_bound_brackets_exact_counts(capfd):
    """MIM_CHECK_BOUNDS=1: every iteration's [lo, hi] from the MFMA bound kernel brackets its exact
    OpenCV inlier count (runKernel + computeError, bit-exact), in chunk 1 (lo and hi) and later chunks,
    on the synthetic workload and on the adversarial sets (near-collinear clusters put points close to
    the horizon of many hypotheses, where OpenCV's own fp32 evaluation is far from the true error)."""
    import os
    import re
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(2, 2, 1200, 2000, 400, inlier_frac=0.1, seed=99)
    os.environ["MIM_CHECK_BOUNDS"] = "1"
    m = Matcher(0)
    try:
        q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
        t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
        m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=6000))
        for s_, d_ in _adversarial_sets():
            m.find_homography(s_, d_, 5.0, 6000)
    finally:
        m.close()
        os.environ.pop("MIM_CHECK_BOUNDS", None)
    cap = capfd.readouterr()
    err = cap.err
    lines = re.findall(r"checked (\d+) lo_viol (\d+) hi_viol (\d+) valid_mismatch (\d+)", err)
    assert lines and sum(int(c) for c, *_ in lines) > 10000
    for c, lo_v, hi_v, vm in lines:
        assert (lo_v, hi_v, vm) == ("0", "0", "0"), err + cap.out


def test_bound_brackets_tight_at_large_n(capfd):
    """Thousands of good matches (n ~ 7,000): the bound kernel's float counts are summed over 32 nt
    values, and a rounding slack that grew with n^2 (round 5: 2.9 counts here) would leave no bracket
    tight (lo == hi) in chunk 1, sending every candidate to the prescreen or the eigensolve.  The slack
    now follows the count itself: the brackets still hold every exact count, and most of chunk 1's are
    tight."""
    import os
    import re
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(1, 1, 8000, 9000, 7000, inlier_frac=0.08, seed=123)
    os.environ["MIM_CHECK_BOUNDS"] = "1"
    m = Matcher(0)
    try:
        q = m.add_set(ds.model_desc[0], ds.model_kp[0])
        t = m.add_set(ds.scene_desc[0], ds.scene_kp[0])
        res = m.match_batch([(q, t)], default_params(max_iters=1500))
    finally:
        m.close()
        os.environ.pop("MIM_CHECK_BOUNDS", None)
    assert int(res[0]["n_good"]) > 4096
    err = capfd.readouterr().err
    lines = re.findall(r"chunk \[(\d+),\d+\): checked (\d+) lo_viol (\d+) hi_viol (\d+) valid_mismatch (\d+) "
                       r"mean_width \S+ tight (\d+)", err)
    assert lines, err
    for c0, c, lo_v, hi_v, vm, tight in lines:
        assert (lo_v, hi_v, vm) == ("0", "0", "0"), err
        if c0 == "0":
            assert int(tight) > 0.1 * int(c), err  # ~20 % at n ~ 7,000 (points between the two diamonds); 0 before


def test_winner_h_reaches_refine(capfd):
    """MIM_WINNER_H=1: the settle pass sends each chunk's largest decided candidate through the exact
    pass, so the refine starts from that candidate's fp64 H.  A candidate the bound kernel pinned
    (lo == hi) used to take the exact kernel's shortcut, which stores no H; it is now
    flagged to run runKernel.  Every problem of the bound path reaches the refine with its bestModel
    (MIM_CHECK_BESTH report), and the records equal MIM_WINNER_H=0's."""
    import os
    import re
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(2, 4, 1200, 2000, 400, inlier_frac=0.1, seed=31337)
    out = {}
    os.environ["MIM_CHECK_BESTH"] = "1"
    try:
        for wh in ("0", "1"):
            os.environ["MIM_WINNER_H"] = wh
            m = Matcher(0)
            try:
                q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
                t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
                res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=20000))
            finally:
                m.close()
            err = capfd.readouterr().err
            rep = re.findall(r"best_h: (\d+) problems with the exact pass's fp64 bestModel, (\d+) without", err)
            assert rep, err
            out[wh] = (res.tobytes(), rep[-1])
    finally:
        os.environ.pop("MIM_CHECK_BESTH", None)
        os.environ.pop("MIM_WINNER_H", None)
    assert out["0"][0] == out["1"][0]
    with_h, without = map(int, out["1"][1])
    assert with_h > 0 and without == 0, out


@pytest.mark.parametrize("mode", ["0", "1"])
def test_sampler_stream_identical(mode):
    """The next chunk's getSubset replay on its own stream (MIM_SAMPLER_STREAM=1, concurrent with
    this chunk's selection kernels, field-level state stores) gives the records and masks of the
    one-stream order, on a workload whose problems terminate early and late."""
    import os
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(2, 4, 1200, 2000, 400, inlier_frac=0.1, seed=31337)
    outs = []
    for m_ in ("0", mode):
        os.environ["MIM_SAMPLER_STREAM"] = m_
        m = Matcher(0)
        try:
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=20000))
            masks = [m.problem_detail(i, int(r["n_good"]))[2] for i, r in enumerate(res)]
            fh = [m.find_homography(s_, d_, 5.0, 20000) + (m.batch_results(1).tobytes(),) for s_, d_ in _adversarial_sets()]
        finally:
            m.close()
            os.environ.pop("MIM_SAMPLER_STREAM", None)
        outs.append((res, masks, fh))
    (r0, m0, f0), (r1, m1, f1) = outs
    assert r0.tobytes() == r1.tobytes()
    for a, b in zip(m0, m1):
        np.testing.assert_array_equal(a, b)
    for (ha, ma, ra), (hb, mb, rb) in zip(f0, f1):
        np.testing.assert_array_equal(ma, mb)
        assert ra == rb


def _small_sets(seed=99):
    """Point sets of 128-300 matches (the chain sampler's range, n >= 128) whose getSubset redraws a
    repeated index every ~20-50 positions, with 20-40 % inliers of a mild homography."""
    rng = np.random.default_rng(seed)
    out = []
    for n in (128, 150, 200, 300):
        src = np.c_[rng.uniform(0, 640, n), rng.uniform(0, 480, n)].astype(np.float32)
        dst = np.c_[rng.uniform(0, 640, n), rng.uniform(0, 480, n)].astype(np.float32)
        k = int(n * rng.uniform(0.2, 0.4))
        dst[:k] = src[:k] * np.float32(1.05) + np.float32(7) + rng.uniform(-0.5, 0.5, (k, 2)).astype(np.float32)
        out.append((src, dst))
    return out


def test_attempt_redraw_list_overflow_equals_walker(oracle):
    """MIM_ATTEMPT_REP_CAP=1: the attempt kernel's per-block list of repeated-index positions holds one
    entry, so nearly every redraw length is resolved in place (the list-overflow path); masks, records
    and H must equal the attempt-by-attempt walker (MIM_SAMPLER_WALK=1) and the oracle."""
    import os
    from computervision_objectdetection_featurematching_amd import Matcher
    sets = _small_sets()
    outs = []
    for env in ({"MIM_ATTEMPT_REP_CAP": "1"}, {"MIM_SAMPLER_WALK": "1"}):
        os.environ.update(env)
        m = Matcher(0)
        try:
            outs.append([m.find_homography(s_, d_, 5.0, 2000) + (m.batch_results(1).tobytes(),) for s_, d_ in sets])
        finally:
            m.close()
            for k in env:
                os.environ.pop(k)
    for (ha, ma, ra), (hb, mb, rb), (s_, d_) in zip(outs[0], outs[1], sets):
        np.testing.assert_array_equal(ma, mb)
        assert ra == rb
        r = oracle.ransac(s_, d_, 5.0, 0.995, 2000)
        np.testing.assert_array_equal(ma, r["mask"])


def test_candidate_prescreen_equals_exact_paths(capfd):
    """The prescreen (closed-form disc test in fp64, MIM_PRESCREEN=1, default) decides a part of the
    candidates without the eigensolve and the settle pass drops those that cannot beat the decided counts
    before them: records and masks identical to the prescreen off, the settle pass off, the largest decided
    candidate sent through the exact pass on every problem (MIM_WINNER_H=1) and to the all-exact
    mode on C4's regime (8 % planted inliers of 2,000 good matches, 50,000 iterations),
    and the debug counts show candidates actually decided."""
    import os
    import re
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(1, 6, 3000, 3000, 2000, inlier_frac=0.08, seed=4242)
    outs = []
    for env in ({"MIM_PRESCREEN": "1", "MIM_DEBUG_NCAND": "1"}, {"MIM_PRESCREEN": "0"}, {"MIM_SETTLE": "0"},
                {"MIM_WINNER_H": "1"}, {"MIM_RANSAC_EXACT": "1"}):
        os.environ.update(env)
        m = Matcher(0)
        try:
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=50000))
            masks = [m.problem_detail(i, int(r["n_good"]))[2] for i, r in enumerate(res)]
        finally:
            m.close()
            for k in env:
                os.environ.pop(k, None)
        outs.append((res, masks))
        if "MIM_DEBUG_NCAND" in env:
            err = capfd.readouterr().err
            lines = re.findall(r"candidates mean ([0-9.]+) max \d+ undecided mean ([0-9.]+)", err)
            assert lines, err[-2000:]
            assert sum(float(a) for a, _ in lines) > 0
            assert sum(float(u) for _, u in lines) < sum(float(a) for a, _ in lines)  # some decided
    (r0, m0) = outs[0]
    assert (r0["status"] == 0).any()
    for r1, m1 in outs[1:]:
        assert r0.tobytes() == r1.tobytes()
        for a, b in zip(m0, m1):
            np.testing.assert_array_equal(a, b)


def test_check_defer_list_equals_in_place():
    """The check rounds' deferred attempts (redraw attempts, samples fp32 cannot decide) decided by
    ransac_check_defer_kernel from the rounds' lists give the same pass bits, hence the same samples and
    records, as deciding them inside the check kernel (MIM_CHECK_DEFER=0), on a C4-shaped batch at
    50,000 iterations and on the adversarial sets; both equal the walker (MIM_SAMPLER_WALK=1)."""
    import os
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    ds = make_dataset(1, 12, 2500, 10000, 2000, inlier_frac=0.08, seed=4242)
    sets = _adversarial_sets()
    outs = []
    for env in ({}, {"MIM_CHECK_DEFER": "0"}, {"MIM_SAMPLER_WALK": "1"}):
        os.environ.update(env)
        m = Matcher(0)
        try:
            q = [m.add_set(d, k) for d, k in zip(ds.model_desc, ds.model_kp)]
            t = [m.add_set(d, k) for d, k in zip(ds.scene_desc, ds.scene_kp)]
            res = m.match_batch([(q[a], t[b]) for a, b in ds.problems], default_params(max_iters=50000))
            fh = [m.find_homography(s_, d_, 5.0, 20000)[1].tobytes() + m.batch_results(1).tobytes()
                  for s_, d_ in sets]
        finally:
            m.close()
            for k in env:
                os.environ.pop(k, None)
        outs.append((res.tobytes(), fh))
    assert outs[0] == outs[1]
    assert outs[0] == outs[2]
