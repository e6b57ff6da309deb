"""Debug: run detect_objects on the first configs[0] scene and save the per-problem records + SIFT."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402
from computervision_objectdetection_featurematching_amd.pipeline import detect_objects, process_model_views  # noqa: E402

with np.load(os.path.join(ROOT, "tests", "golden", "c1_sugar_box.npz")) as z:
    d = {k: z[k] for k in z.files}
names = sorted(k[5:] for k in d if k.startswith("view/"))
m = Matcher(0)
model = process_model_views(m, "004_sugar_box", [(d[f"view/{n}"], d[f"mask/{n}"]) for n in names])
sid = sorted(k[8:] for k in d if k.startswith("exp/res/"))[0]
run = detect_objects(m, d[f"scene/{sid}"], [model], keep=True)
out = {"res": np.stack([run.results["n_good"], run.results["n_inl"], run.results["status"], run.results["iters"]], 1),
       "H": run.results["H"]}
for i in range(len(names)):
    out[f"vk{i}"] = model.keypoints[i]
    out[f"vd{i}"] = model.descriptors[i]
for s in range(5):
    out[f"sk{s}"] = run.scene_kp[s]
    out[f"sd{s}"] = run.scene_desc[s]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "c1_dump.npz"), **out)
print("ok", sid)
