"""Debug: exact-mode RANSAC trace of one saved problem (MIM_RANSAC_EXACT=1 MIM_DEBUG_TRACE=1)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402

z = np.load(os.path.join(ROOT, "tools", "c1_bad_problems.npz"))
m = Matcher(0)
i = sys.argv[1]
H, mask = m.find_homography(z["src" + i], z["dst" + i])
print("done", i, file=sys.stderr)
m.close()
