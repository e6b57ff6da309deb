"""Times the GPU SIFT / resize / detectObjects path on configs[0] data (tests/golden/c1_sugar_box.npz).

python tools/time_sift.py [--reps N] [--oracle]   (prints one JSON line)"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--oracle", action="store_true")
    a = ap.parse_args()
    from computervision_objectdetection_featurematching_amd import Matcher
    from computervision_objectdetection_featurematching_amd.pipeline import SCALES, detect_objects, process_model_views
    with np.load(os.path.join(ROOT, "tests", "golden", "c1_sugar_box.npz")) as z:
        d = {k: z[k] for k in z.files if not k.startswith("exp/")}
    names = sorted(k[5:] for k in d if k.startswith("view/"))
    scene = d[sorted(k for k in d if k.startswith("scene/"))[0]]
    m = Matcher(0)
    out = {}
    m.sift_detect_compute(scene)  # warm-up (workspace allocation, code load)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        k, _ = m.sift_detect_compute(scene)
    out["sift_640x480_ms"] = (time.perf_counter() - t0) / a.reps * 1e3
    out["sift_640x480_kp"] = len(k)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        for s in SCALES:
            m.sift_detect_compute(m.resize_linear(scene, fx=s))
    out["scene_5_scales_ms"] = (time.perf_counter() - t0) / a.reps * 1e3
    t0 = time.perf_counter()
    model = process_model_views(m, "004_sugar_box", [(d[f"view/{n}"], d[f"mask/{n}"]) for n in names])
    out["model_29_views_ms"] = (time.perf_counter() - t0) * 1e3
    detect_objects(m, scene, [model])
    t0 = time.perf_counter()
    for _ in range(a.reps):
        dets = detect_objects(m, scene, [model])
    out["detect_objects_ms"] = (time.perf_counter() - t0) / a.reps * 1e3
    out["detections"] = dets
    if a.oracle:
        from oracle import oracle as O
        t0 = time.perf_counter()
        O.sift_detect_compute(scene)
        out["oracle_sift_640x480_ms"] = (time.perf_counter() - t0) * 1e3
    m.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
