"""Fraction of RANSAC hypotheses that are "front-facing" on the C4 workload: W = h6 x + h7 y + h8 of the
same sign over the source points' bounding box (W is affine in (x, y), so its sign at the 4 corners
decides every point), the condition for the linearised bound C W + E - |ex|.

Problem shape of BASELINE configs[3] (synthetic.py): 2,000 good matches, 8 % at H_true(p) + U(+-0.5 px),
the rest random scene positions; samples = random 4-subsets passing checkSubset's orientation test
(fp64, as fundam.cpp), H by the normalised DLT (numpy SVD).  Prints the fractions over `--samples`.

usage: python3 tools/front_facing.py [--samples 200000] [--seed 1]
"""
import argparse
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from computervision_objectdetection_featurematching_amd import synthetic as S  # noqa: E402


def dlt(src, dst):
    A = []
    for (x, y), (u, v) in zip(src, dst):
        A.append([x, y, 1, 0, 0, 0, -u * x, -u * y, -u])
        A.append([0, 0, 0, x, y, 1, -v * x, -v * y, -v])
    _, _, vt = np.linalg.svd(np.asarray(A))
    h = vt[-1]
    return h / h[8] if abs(h[8]) > 1e-300 else h


def orient_ok(src, dst):
    tt = ((0, 1, 2), (1, 2, 3), (0, 2, 3), (0, 1, 3))
    neg = 0
    for a, b, c in tt:
        da = np.linalg.det(np.array([[*src[a], 1], [*src[b], 1], [*src[c], 1]]))
        db = np.linalg.det(np.array([[*dst[a], 1], [*dst[b], 1], [*dst[c], 1]]))
        neg += da * db < 0
    return neg in (0, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=200000)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    n, n_in = 2000, 160
    src = np.stack([rng.uniform(0, S.IMG_W, n), rng.uniform(0, S.IMG_H, n)], 1)
    H = S.random_homography(rng)
    dst = np.stack([rng.uniform(0, S.IMG_W, n), rng.uniform(0, S.IMG_H, n)], 1)
    dst[:n_in] = S.apply_h(H, src[:n_in]) + rng.uniform(-0.5, 0.5, (n_in, 2))
    lo, hi = src.min(0), src.max(0)
    corners = np.array([[lo[0], lo[1]], [lo[0], hi[1]], [hi[0], lo[1]], [hi[0], hi[1]]])
    tried = passed = front = 0
    w_pos_pairs = 0.0
    while passed < a.samples:
        idx = rng.choice(n, 4, replace=False)
        tried += 1
        if not orient_ok(src[idx], dst[idx]):
            continue
        passed += 1
        h = dlt(src[idx], dst[idx])
        w = corners @ h[6:8] + h[8]
        front += bool(np.all(w > 0) or np.all(w < 0))
        wp = src @ h[6:8] + h[8]
        w_pos_pairs += max(np.mean(wp > 0), np.mean(wp < 0))
    print(f"samples {passed} (checkSubset orientation pass rate {passed / tried:.3f})")
    print(f"front-facing over the bounding box: {front / passed:.4f}")
    print(f"mean fraction of points on the majority side of the horizon: {w_pos_pairs / passed:.4f}")


if __name__ == "__main__":
    main()
