"""Re-run chosen corpus cases (tests/test_bounds_corpus_gpu.py) with MIM_CHECK_BOUNDS=1 and print the
device's violation details.  usage: python tools/bound_violation_probe.py big_persp:14 big_persp:16"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["MIM_CHECK_BOUNDS"] = "1"

from computervision_objectdetection_featurematching_amd import Matcher  # noqa: E402
import test_bounds_corpus_gpu as T  # noqa: E402

m = Matcher(0)
for arg in sys.argv[1:]:
    fam, seed = arg.split(":")
    src, dst, iters = T._family(fam, int(seed))
    print(f"== {fam}:{seed} n={len(src)} iters={iters}", flush=True)
    m.find_homography(src, dst, 5.0, iters, 0.999999999)
    m.synchronize()
    sys.stdout.flush()
m.close()
