"""Diagnostic (round 5ai): the bounds corpus (tests/test_bounds_corpus_gpu.py) through find_homography in
the filtered mode with the prescreen's debug recount (MIM_CHECK_PRESCREEN=1), and the filtered records
against the all-exact mode, per family; prints the families/seeds that differ and the mismatch lines."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import test_bounds_corpus_gpu as T  # noqa: E402
from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402

corpus = T._corpus()
outs = []
for mode in ("0", "1"):
    os.environ["MIM_RANSAC_EXACT"] = mode
    if mode == "0":
        os.environ["MIM_CHECK_PRESCREEN"] = "1"
    m = Matcher(0)
    o = []
    for fam, seed, src, dst, iters in corpus:
        H, mask = m.find_homography(src, dst, 5.0, iters, 0.995)
        o.append((fam, seed, None if H is None else H.tobytes(), mask.tobytes(), m.batch_results(1).tobytes()))
    m.close()
    os.environ.pop("MIM_CHECK_PRESCREEN", None)
    outs.append(o)
diff = [a[:2] for a, b in zip(*outs) if a != b]
print("differ:", len(diff), diff[:20], flush=True)
