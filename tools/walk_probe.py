"""Diagnostic: find_homography on the saved slow dataset problems (gpurun_out/ds_slow.npz)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402

z = np.load(os.path.join(ROOT, "tests", "golden", "ds_small_problems.npz"))
m = Matcher(0)
m.set_timing(True)
for k in sorted(z.files):
    if k.startswith("src"):
        m.find_homography(z[k], z["dst" + k[3:]])
        r = m.batch_results(1)
        print(k, int(r["iters"][0]), m.kernel_ms("sample"), m.kernel_ms("chain"), flush=True)
m.close()
