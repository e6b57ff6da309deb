"""Host-side phase times of one c1img scene through the pipeline's calls (diagnostic).

python tools/scene_host_probe.py [--scenes N]

Runs detect_objects' steps one by one on configs[0] data (tests/golden/c1_sugar_box.npz), kernel timing
off, and prints the median wall time of each (us): sift (mim_sift_scales_sets, returns once the sets
are registered), probs (the problem array), enqueue (mim_batch_run returning), wait (mim_batch_results:
the batch's device work), gather (inlier points), boxes.  Which of them the GPU idles through is what
the single-scene latency can still lose on the host.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=30)
    a = ap.parse_args()
    from computervision_objectdetection_featurematching_amd import Matcher
    from computervision_objectdetection_featurematching_amd.pipeline import (SCALES, _model_sets, detect_boxes,
                                                                           process_model_views)
    with np.load(os.path.join(ROOT, "tests", "golden", "c1_sugar_box.npz")) as z:
        d = {k: z[k] for k in z.files if not k.startswith("exp/")}
    names = sorted(k[5:] for k in d if k.startswith("view/"))
    scenes = [d[k] for k in sorted(k for k in d if k.startswith("scene/"))]
    m = Matcher(0)
    m.set_timing(False)
    model = process_model_views(m, "004_sugar_box", [(d[f"view/{n}"], d[f"mask/{n}"]) for n in names])
    ph = {k: [] for k in ("sets", "sift", "probs", "enqueue", "wait", "gather", "boxes", "total")}
    for i in range(a.scenes + 3):
        scene = scenes[i % len(scenes)]
        t0 = time.perf_counter()
        view_ids = _model_sets(m, [model])
        t1 = time.perf_counter()
        scene_ids, _, _ = m.sift_scales_to_sets(scene, SCALES)
        t2 = time.perf_counter()
        sid = np.asarray(scene_ids, np.int32)
        v = np.asarray(view_ids[0], np.int32)
        probs = np.stack([np.tile(v, len(SCALES)), np.repeat(sid, len(v))], axis=1)
        psc = np.repeat(np.asarray(SCALES, np.float32), len(v))
        t3 = time.perf_counter()
        n = m.match_batch_async(probs)
        t4 = time.perf_counter()
        m.batch_results(n)
        t5 = time.perf_counter()
        offs, pts = m.batch_inlier_points(n, psc)
        t6 = time.perf_counter()
        detect_boxes(pts[offs[0]:offs[n]].copy())
        t7 = time.perf_counter()
        if i < 3:
            continue
        for k, (s, e) in zip(("sets", "sift", "probs", "enqueue", "wait", "gather", "boxes", "total"),
                             ((t0, t1), (t1, t2), (t2, t3), (t3, t4), (t4, t5), (t5, t6), (t6, t7), (t0, t7))):
            ph[k].append(1e6 * (e - s))
    print({k: round(float(np.median(v)), 1) for k, v in ph.items()})
    m.close()


if __name__ == "__main__":
    main()
