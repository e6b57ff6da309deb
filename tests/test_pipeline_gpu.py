"""BASELINE.json configs[0] end to end on the reference's own data, on the GPU: the sugar_box model (29
views with masks, ModelsDetector.cpp:46-80) against its test views through detectObjects
(TestsDetector.cpp:32-251): resize + SIFT per scale on the GPU, the 145 (scale, view) problems as one
device batch, the boxes in the library's host stage — every stage against the CPU restatement's
outputs committed in tests/golden/c1_sugar_box.npz (tests/golden/make_c1_golden.py).

Bar: SIFT keypoints + descriptors identical (sha256), per-problem n_good / n_inl / status / iters
identical, H bit-identical (the refit and LM run in the oracle's operation order), the model's
allUnfilteredScenePts identical, detections identical.
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SCALES = (0.7, 0.85, 1.0, 1.15, 1.3)


def sift_hash(k, d):
    return np.frombuffer(hashlib.sha256(k.tobytes() + np.ascontiguousarray(d, np.float32).tobytes()).digest(), np.uint8)


@pytest.fixture(scope="module")
def c1():
    with np.load(os.path.join(HERE, "golden", "c1_sugar_box.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def model(matcher, c1):
    from computervision_objectdetection_featurematching_amd.pipeline import process_model_views
    names = sorted(k[5:] for k in c1 if k.startswith("view/"))
    m = process_model_views(matcher, "004_sugar_box", [(c1[f"view/{n}"], c1[f"mask/{n}"]) for n in names])
    return names, m


def test_model_views_sift(model, c1):
    names, m = model
    assert len(names) == 29
    bad = [n for n, k, d in zip(names, m.keypoints, m.descriptors) if not np.array_equal(sift_hash(k, d), c1[f"exp/sift/view/{n}"])]
    assert not bad, f"SIFT differs on views {bad}"


def test_detect_objects_matches_oracle(matcher, model, c1):
    from computervision_objectdetection_featurematching_amd.pipeline import detect_objects
    _, m = model
    scenes = sorted(k[8:] for k in c1 if k.startswith("exp/res/"))
    assert len(scenes) >= 3
    for sid in scenes:
        run = detect_objects(matcher, c1[f"scene/{sid}"], [m], keep=True, keep_descriptors=True)
        for s, k, d in zip(SCALES, run.scene_kp, run.scene_desc):
            assert np.array_equal(sift_hash(k, d), c1[f"exp/sift/{sid}/{s}"]), (sid, s)
        r = run.results
        got = np.stack([r["n_good"], r["n_inl"], r["status"], r["iters"]], 1)
        np.testing.assert_array_equal(got, c1[f"exp/res/{sid}"], err_msg=sid)
        Ho = c1[f"exp/H/{sid}"]
        ok = np.isin(r["status"], (0, 3, 4))  # RANSAC ran and found a model
        np.testing.assert_array_equal(r["H"][ok], Ho[ok], err_msg=sid)
        np.testing.assert_array_equal(run.points[0], c1[f"exp/pts/{sid}"], err_msg=sid)
        boxes = np.array([b for b, _ in run.detections], np.int32).reshape(-1, 4)
        np.testing.assert_array_equal(boxes, c1[f"exp/boxes/{sid}"], err_msg=sid)
        assert all(n == "004_sugar_box" for _, n in run.detections)


def test_detect_objects_unlabelled_scenes_run(matcher, model, c1):
    """The other test views: the pipeline runs and is repeatable (same detections twice)."""
    from computervision_objectdetection_featurematching_amd.pipeline import detect_objects
    _, m = model
    scenes = sorted(k[6:] for k in c1 if k.startswith("scene/"))
    for sid in scenes[3:6]:
        a = detect_objects(matcher, c1[f"scene/{sid}"], [m])
        b = detect_objects(matcher, c1[f"scene/{sid}"], [m])
        assert a == b


def test_scenes_in_flight_identical(c1):
    """Several scenes at once, one library context and host thread each (as bench.py --config c1img
    runs them): every scene's records, H bits, scene points and boxes equal the golden run's."""
    from concurrent.futures import ThreadPoolExecutor

    from computervision_objectdetection_featurematching_amd import Matcher
    from computervision_objectdetection_featurematching_amd.pipeline import detect_objects, process_model_views
    names = sorted(k[5:] for k in c1 if k.startswith("view/"))
    views = [(c1[f"view/{n}"], c1[f"mask/{n}"]) for n in names]
    scenes = sorted(k[8:] for k in c1 if k.startswith("exp/res/"))
    ms = [Matcher(0) for _ in scenes]
    try:
        model = process_model_views(ms[0], "004_sugar_box", views)  # host arrays, shared by the contexts

        def one(k):
            return [detect_objects(ms[k], c1[f"scene/{scenes[k]}"], [model], keep=True) for _ in range(2)]

        with ThreadPoolExecutor(len(scenes)) as pool:
            runs = list(pool.map(one, range(len(scenes))))
        for sid, pair in zip(scenes, runs):
            for run in pair:
                r = run.results
                got = np.stack([r["n_good"], r["n_inl"], r["status"], r["iters"]], 1)
                np.testing.assert_array_equal(got, c1[f"exp/res/{sid}"], err_msg=sid)
                ok = np.isin(r["status"], (0, 3, 4))
                np.testing.assert_array_equal(r["H"][ok], c1[f"exp/H/{sid}"][ok], err_msg=sid)
                np.testing.assert_array_equal(run.points[0], c1[f"exp/pts/{sid}"], err_msg=sid)
                boxes = np.array([b for b, _ in run.detections], np.int32).reshape(-1, 4)
                np.testing.assert_array_equal(boxes, c1[f"exp/boxes/{sid}"], err_msg=sid)
    finally:
        for mm in ms:
            mm.close()
