"""The reference's whole run on its own data, on the GPU (main.cpp:17-33): the three objects' models
(ModelsDetector.cpp:46-80, 89 views with masks) against all 30 test images through detectObjects
(TestsDetector.cpp:32-251), the results files (Output.cpp:15-57, utils.cpp:12-20) and the metrics
(metrics.cpp) — against the CPU restatement's run committed in tests/golden/dataset_expected.json
(tests/golden/make_dataset_golden.py; objects and views in sorted order, the reference's order being
filesystem-dependent).

Bar: every scene's detections (boxes and model names, in order) and every model's number of inlier
scene points identical; mean IoU, per-class IoU and per-class accuracy of the results files identical
to the bit (computed by include/mim_detect.hpp through tests/cpp/test_detect.cpp).
"""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def data():
    with np.load(os.path.join(HERE, "golden", "dataset_gray.npz")) as z:
        imgs = {k: z[k] for k in z.files}
    with open(os.path.join(HERE, "golden", "dataset_expected.json")) as f:
        exp = json.load(f)
    return imgs, exp


def test_dataset_end_to_end(matcher, data, tmp_path):
    from computervision_objectdetection_featurematching_amd.pipeline import (process_all_test_images,
                                                                              process_model_views)
    imgs, exp = data
    objs = sorted({k.split("/")[0] for k in imgs})
    models = []
    for obj in objs:
        views = sorted(k for k in imgs if k.startswith(f"{obj}/view/"))
        models.append(process_model_views(matcher, obj, [(imgs[k], imgs.get(k.replace("/view/", "/mask/")))
                                                         for k in views]))
    scenes = [(obj, k.split("/")[-1] + "-color", imgs[k]) for obj in objs
              for k in sorted(k for k in imgs if k.startswith(f"{obj}/scene/"))]
    out = tmp_path / "output"
    got = process_all_test_images(matcher, scenes, models, str(out))
    assert len(got) == len(exp["scenes"]) == 30
    bad = []
    for (folder, name), dets in got.items():
        e = exp["scenes"][f"{folder}/{name[:-6]}"]
        if [[*b, n] for b, n in dets] != e["detections"]:
            bad.append((folder, name, dets, e["detections"]))
    assert not bad, bad[:3]
    # the metrics of the results files (the product header through the C++ test driver)
    drv = str(tmp_path / "test_detect")
    subprocess.check_call(["g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "test_detect.cpp"), "-o", drv])
    r = subprocess.run([drv, "metrics", os.path.join(HERE, "golden", "dataset"), str(out)], capture_output=True,
                       text=True, check=True)
    vals = {" ".join(line.split()[:-1]): float.fromhex(line.split()[-1]) for line in r.stdout.splitlines()}
    # class IoU and accuracy bit for bit; the mean is a float sum over the class folders in directory
    # order (metrics.cpp:12-26, filesystem-dependent, as in the reference): any order of the same sum
    assert {k: v for k, v in vals.items() if k != "mean_iou"} == {k: v for k, v in exp["metrics"].items() if k != "mean_iou"}
    import itertools
    ious = [np.float32(v) for k, v in vals.items() if k.startswith("class_iou")]
    means = set()
    for perm in itertools.permutations(ious):
        acc = np.float32(0)
        for v in perm:
            acc = np.float32(acc + v)
        means.add(float(np.float32(acc / np.float32(len(ious)))))
    assert vals["mean_iou"] in means and exp["metrics"]["mean_iou"] in means
    print("mean IoU", vals["mean_iou"], {k: v for k, v in vals.items() if k.startswith("accuracy")})


def test_dataset_scenes_in_flight(data, tmp_path):
    """The same run with 3 scenes in flight (3 contexts, one host thread each, scene i on context
    i mod 3): every scene's detections equal the oracle run's."""
    from computervision_objectdetection_featurematching_amd import Matcher
    from computervision_objectdetection_featurematching_amd.pipeline import (process_all_test_images,
                                                                              process_model_views)
    imgs, exp = data
    objs = sorted({k.split("/")[0] for k in imgs})
    ms = [Matcher(0) for _ in range(3)]
    try:
        models = [process_model_views(ms[0], obj, [(imgs[k], imgs.get(k.replace("/view/", "/mask/")))
                                                   for k in sorted(k for k in imgs if k.startswith(f"{obj}/view/"))])
                  for obj in objs]
        scenes = [(obj, k.split("/")[-1] + "-color", imgs[k]) for obj in objs
                  for k in sorted(k for k in imgs if k.startswith(f"{obj}/scene/"))]
        got = process_all_test_images(ms, scenes, models, str(tmp_path / "output"))
        assert list(got) == [(f, n) for f, n, _ in scenes]
        bad = [(f, n) for (f, n), dets in got.items()
               if [[*b, nm] for b, nm in dets] != exp["scenes"][f"{f}/{n[:-6]}"]["detections"]]
        assert not bad, bad[:3]
        for f, n, _ in scenes:
            assert (tmp_path / "output" / f / f"{n}_results.txt").exists()
    finally:
        for mm in ms:
            mm.close()
