"""The reference's whole run (main.cpp:17-33) on its own data on one MI355X, timed: models
(processAllModelsImages), every test image (processAllTestImages: detectObjects + results files), then
the metrics of the results files (include/mim_detect.hpp through tests/cpp/test_detect.cpp).

python tools/run_dataset.py [out_dir]   -> one JSON line (timings, mean IoU, accuracies, parity vs
tests/golden/dataset_expected.json, the CPU restatement's run)."""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from computervision_objectdetection_featurematching_amd import Matcher
    from computervision_objectdetection_featurematching_amd.pipeline import process_all_test_images, process_model_views
    out_dir = sys.argv[1] if len(sys.argv) > 1 else tempfile.mkdtemp()
    with np.load(os.path.join(ROOT, "tests", "golden", "dataset_gray.npz")) as z:
        imgs = {k: z[k] for k in z.files}
    with open(os.path.join(ROOT, "tests", "golden", "dataset_expected.json")) as f:
        exp = json.load(f)
    objs = sorted({k.split("/")[0] for k in imgs})
    nf = int(os.environ.get("MIM_SCENES_IN_FLIGHT", "3"))  # contexts, one host thread each
    m = Matcher(0)
    extra = [Matcher(0) for _ in range(nf - 1)]
    # warm-up (code objects, workspaces) on one view and one scene, outside the timings
    any_view = sorted(k for k in imgs if "/view/" in k)[0]
    warm = process_model_views(m, "warm", [(imgs[any_view], None)])
    process_all_test_images(m, [(objs[0], "warm", imgs[sorted(k for k in imgs if "/scene/" in k)[0]])], [warm],
                            tempfile.mkdtemp())
    t0 = time.perf_counter()
    models = []
    for obj in objs:
        views = sorted(k for k in imgs if k.startswith(f"{obj}/view/"))
        models.append(process_model_views(m, obj, [(imgs[k], imgs.get(k.replace("/view/", "/mask/"))) for k in views]))
    t1_models = time.perf_counter()
    # warm the other contexts (code objects, workspaces, the models' sets), timed apart
    for mm in extra:
        process_all_test_images(mm, [(objs[0], "warm", imgs[sorted(k for k in imgs if "/scene/" in k)[0]])], models,
                                tempfile.mkdtemp())
    t1b = time.perf_counter()
    scenes = [(obj, k.split("/")[-1] + "-color", imgs[k]) for obj in objs
              for k in sorted(k for k in imgs if k.startswith(f"{obj}/scene/"))]
    t1 = time.perf_counter()
    got = process_all_test_images([m, *extra], scenes, models, out_dir)
    t2 = time.perf_counter()
    mism = sum([[*b, n] for b, n in d] != exp["scenes"][f"{f}/{s[:-6]}"]["detections"] for (f, s), d in got.items())
    drv = os.path.join(tempfile.mkdtemp(), "test_detect")
    subprocess.check_call(["g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "test_detect.cpp"), "-o", drv])
    r = subprocess.run([drv, "metrics", os.path.join(ROOT, "tests", "golden", "dataset"), out_dir], capture_output=True,
                       text=True, check=True)
    vals = {" ".join(line.split()[:-1]): float.fromhex(line.split()[-1]) for line in r.stdout.splitlines()}
    n_views = sum(len(mm.descriptors) for mm in models)
    print(json.dumps({
        "models": {"objects": len(models), "views": n_views, "seconds": round(t1_models - t0, 4),
                   "other_contexts_setup_seconds": round(t1b - t1_models, 4)},
        "scenes": {"n": len(scenes), "problems_per_scene": 5 * n_views, "in_flight": nf,
                   "seconds": round(t2 - t1, 4), "ms_per_scene": round(1e3 * (t2 - t1) / len(scenes), 2)},
        "metrics": vals,
        # the mean is summed in the class folders' directory order (filesystem-dependent): compare the rest
        "class_metrics_equal_to_oracle_run": {k: v for k, v in vals.items() if k != "mean_iou"} ==
                                             {k: v for k, v in exp["metrics"].items() if k != "mean_iou"},
        "scenes_with_detections_differing_from_oracle_run": int(mism)}))
    m.close()


if __name__ == "__main__":
    main()
