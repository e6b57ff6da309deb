"""Diagnostic: per-problem sampler time on one scene of the full dataset (all models); saves the three
slowest match sets to gpurun_out/ds_slow.npz (copied to tests/golden/ds_small_problems.npz)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402
from computervision_objectdetection_featurematching_amd.pipeline import SCALES, detect_objects, process_model_views  # noqa: E402

with np.load(os.path.join(ROOT, "tests", "golden", "dataset_gray.npz")) as z:
    imgs = {k: z[k] for k in z.files}
objs = sorted({k.split("/")[0] for k in imgs})
m = Matcher(0)
models = [process_model_views(m, o, [(imgs[k], imgs.get(k.replace("/view/", "/mask/")))
                                     for k in sorted(k for k in imgs if k.startswith(f"{o}/view/"))]) for o in objs]
scene_keys = sorted(k for k in imgs if "/scene/" in k)
sk = scene_keys[int(sys.argv[1]) if len(sys.argv) > 1 else 0]
m.set_timing(True)
run = detect_objects(m, imgs[sk], models, keep=True)
r = run.results
print(json.dumps({"scene": sk, "sample_ms": m.kernel_ms("sample"), "chain_ms": m.kernel_ms("chain")}))
tags = [(mi, si, vi) for mi in range(len(models)) for si in range(len(SCALES)) for vi in range(len(models[mi].descriptors))]
sets = []
for i, (mi, si, vi) in enumerate(tags):
    ng = int(r["n_good"][i])
    if ng < 5:
        continue
    q, t, _ = m.problem_detail(i, ng)
    vk = models[mi].keypoints[vi]
    src = np.stack([vk["x"], vk["y"]], 1)[q]
    dst = np.stack([run.scene_kp[si]["x"], run.scene_kp[si]["y"]], 1)[t]
    sets.append((i, ng, src, dst))
per = []
for i, ng, src, dst in sets:
    m.find_homography(src, dst)
    res = m.batch_results(1)
    per.append((i, ng, int(res["iters"][0]), int(res["status"][0]), round(m.kernel_ms("sample"), 3),
                round(m.kernel_ms("chain"), 3), len(np.unique(dst, axis=0)), len(np.unique(src, axis=0))))
per.sort(key=lambda x: -x[4])
print(json.dumps(per[:10]))
slow = {}
for i, ng, src, dst in sets:
    if i in [x[0] for x in per[:3]]:
        slow[f"src{i}"] = src
        slow[f"dst{i}"] = dst
np.savez(os.path.join(ROOT, "gpurun_out", "ds_slow.npz"), **slow)
