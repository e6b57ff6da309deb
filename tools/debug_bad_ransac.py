"""Debug: mim_find_homography on saved point sets (tools/c1_bad_problems.npz); prints iters / n_inl."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402

z = np.load(os.path.join(ROOT, "tools", "c1_bad_problems.npz"))
m = Matcher(0)
for k in sorted(z.files):
    if not k.startswith("src"):
        continue
    i = k[3:]
    H, mask = m.find_homography(z[k], z["dst" + i])
    res = m.batch_results(1)
    print(os.environ.get("MIM_RANSAC_EXACT", "0"), i, int(res["n_inl"][0]), int(res["iters"][0]), int(res["status"][0]),
          None if H is None else float(H[2, 2]))
m.close()
