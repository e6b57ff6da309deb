"""Round 3bg diagnosis: the reference's sugar_box scenes through detect_objects with the chunk-2 x-half
prefilter (MIM_BOUND_XPRE=1) and without (0), one context, sequentially; prints the records that differ
from the golden run and the per-chunk candidate counts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402
from computervision_objectdetection_featurematching_amd.pipeline import detect_objects, process_model_views  # noqa: E402

with np.load(os.path.join(ROOT, "tests", "golden", "c1_sugar_box.npz")) as z:
    c1 = {k: z[k] for k in z.files}
names = sorted(k[5:] for k in c1 if k.startswith("view/"))
scenes = sorted(k[8:] for k in c1 if k.startswith("exp/res/"))
m = Matcher(0)
model = process_model_views(m, "004_sugar_box", [(c1[f"view/{n}"], c1[f"mask/{n}"]) for n in names])
for x in ("0", "1", "0", "1"):
    os.environ["MIM_BOUND_XPRE"] = x
    for sid in scenes:
        r = detect_objects(m, c1[f"scene/{sid}"], [model], keep=True).results
        got = np.stack([r["n_good"], r["n_inl"], r["status"], r["iters"]], 1)
        exp = c1[f"exp/res/{sid}"]
        bad = np.nonzero((got != exp).any(1))[0]
        print("xpre", x, sid, "mismatched problems", bad.tolist()[:10],
              [(got[i].tolist(), exp[i].tolist()) for i in bad[:4]], flush=True)
m.close()
