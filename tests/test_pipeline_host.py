"""CPU checks of the pipeline's host pieces: the C-ABI box stage (mim_detect_boxes) against the
oracle's clustering (oracle/detect_oracle.py) on the golden allUnfilteredScenePts of configs[0]
(tests/golden/c1_sugar_box.npz), and the results-file format (utils.cpp:12-20).  No GPU calls."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def c1():
    with np.load(os.path.join(HERE, "golden", "c1_sugar_box.npz")) as z:
        return {k: z[k] for k in z.files if k.startswith("exp/")}


def test_detect_boxes_cabi_matches_golden(c1):
    from computervision_objectdetection_featurematching_amd import build
    build.build()
    from computervision_objectdetection_featurematching_amd.pipeline import detect_boxes
    for key in [k for k in c1 if k.startswith("exp/pts/")]:
        sid = key[8:]
        got = np.array(detect_boxes(c1[key]), np.int32).reshape(-1, 4)
        np.testing.assert_array_equal(got, c1[f"exp/boxes/{sid}"])


def test_detect_boxes_edge_cases():
    from computervision_objectdetection_featurematching_amd.pipeline import default_box_params, detect_boxes
    assert detect_boxes(np.zeros((0, 2), np.float32)) == []
    few = np.random.default_rng(0).uniform(0, 10, (17, 2)).astype(np.float32)  # < MIN_POINTS_PER_CLUSTER
    assert detect_boxes(few) == []
    blob = np.random.default_rng(1).uniform(100, 110, (40, 2)).astype(np.float32)  # box area < 2500
    assert detect_boxes(blob) == []
    assert len(detect_boxes(blob, default_box_params(min_box_area=1))) == 1


def test_save_detections_format(tmp_path):
    from computervision_objectdetection_featurematching_amd.pipeline import save_detections
    p = tmp_path / "r.txt"
    save_detections(str(p), [((10, 20, 30, 40), "004_sugar_box"), ((1, 2, 3, 4), "035_power_drill")])
    assert p.read_text() == "004_sugar_box 10 20 40 60\n035_power_drill 1 2 4 6\n"


def test_scene_run_descriptors_only_when_kept():
    from computervision_objectdetection_featurematching_amd.pipeline import SceneRun
    run = SceneRun([], None, np.zeros(0), [], [])
    with pytest.raises(ValueError, match="keep_descriptors"):
        run.descriptors()
    assert run.scene_desc is None
    d = [np.zeros((2, 128), np.float32)]
    assert SceneRun([], d, np.zeros(0), [], []).descriptors() is d
    assert SceneRun(scene_kp=[], scene_desc=d, results=np.zeros(0), points=[], detections=[]).scene_desc is d
