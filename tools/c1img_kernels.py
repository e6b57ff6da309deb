"""Diagnostic: per-kernel device time of one configs[0] real-image batch (detect_objects), HIP events."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402
from computervision_objectdetection_featurematching_amd.pipeline import detect_objects, process_model_views  # noqa: E402

with np.load(os.path.join(ROOT, "tests", "golden", "c1_sugar_box.npz")) as z:
    d = {k: z[k] for k in z.files if not k.startswith("exp/")}
names = sorted(k[5:] for k in d if k.startswith("view/"))
m = Matcher(0)
model = process_model_views(m, "004_sugar_box", [(d[f"view/{n}"], d[f"mask/{n}"]) for n in names])
scene = d[sorted(k for k in d if k.startswith("scene/"))[0]]
detect_objects(m, scene, [model])
m.set_timing(True)
t0 = time.perf_counter()
run = detect_objects(m, scene, [model], keep=True)
el = time.perf_counter() - t0
ks = ("knn", "ratio", "attempt", "chain", "check", "sample", "score", "cand", "exact", "select", "refine")
out = {"wall_ms": el * 1e3, "kernels_ms": {k: m.kernel_ms(k) for k in ks}}
r = run.results
out["n_good"] = r["n_good"].tolist()
out["iters"] = r["iters"].tolist()
print(json.dumps(out))

# per problem: RANSAC alone on its good matches, sample-kernel time (details first: a primitive call
# replaces the ctx's last batch)
sets = []
for i in range(len(r)):
    ng = int(r["n_good"][i])
    if ng < 5:
        continue
    q, t, _ = m.problem_detail(i, ng)
    si, vi = i // len(names), i % len(names)
    src = np.stack([model.keypoints[vi]["x"], model.keypoints[vi]["y"]], 1)[q]
    dst = np.stack([run.scene_kp[si]["x"], run.scene_kp[si]["y"]], 1)[t]
    sets.append((i, ng, src, dst))
per = []
for i, ng, src, dst in sets:
    m.find_homography(src, dst)
    res = m.batch_results(1)
    per.append((i, ng, int(res["iters"][0]), round(m.kernel_ms("sample"), 3), round(m.kernel_ms("chain"), 3),
                len(np.unique(dst, axis=0)), len(np.unique(src, axis=0))))
per.sort(key=lambda x: -x[3])
print(json.dumps(per[:12]))
slow = {f"src{i}": src for i, ng, src, dst in sets if i in [x[0] for x in per[:4]]}
slow.update({f"dst{i}": dst for i, ng, src, dst in sets if i in [x[0] for x in per[:4]]})
np.savez(os.path.join(ROOT, "gpurun_out", "c1_slow.npz"), **slow)
