"""How often would an Eigen-built OpenCV differ from the restatement?  (VERDICT r1 "next" item 5)

OpenCV built HAVE_EIGEN (Ubuntu 22.04's libopencv 4.5.4 is) solves the 9x9 eigenproblem of every
`runKernel` (fundam.cpp HomographyEstimatorCallback) with Eigen's SelfAdjointEigenSolver, while the
oracle and the GPU restate OpenCV's own JacobiImpl_.  Both are backward stable, so their
minimal-sample models differ by a few ulp.  This study perturbs every minimal-sample model of the
oracle's RANSAC by a pseudo-random k in [-u, u] ulp per element (oracle knob
orc_set_model_perturbation) and counts, against the unperturbed run, the problems whose RANSAC best
mask, iteration count, best iteration, findHomography status or final mask change, the largest
relative change of the final (refined) H, and how many of all evaluated hypotheses got a different
inlier count (the per-hypothesis flip rate behind any outcome change).

Point sets have the shapes of the BASELINE configs' RANSAC inputs:
  c1: 145 problems, 10-300 good matches, 20-80 % inliers, maxIters 2000 (the reference's own run)
  c2: 40 problems, 400 good matches, 8 % inliers, maxIters 2000
  c3: 16 problems, 2000 good matches, 8 % inliers, maxIters 50000
Model points uniform in 640x480, inliers at H(model) + U(+-0.5 px), outliers uniform.

Levels 2^12, 2^20 and 2^28 ulp (relative ~1e-12, 2e-10, 6e-8) show that the knob bites and how the
flip rate grows with the disagreement.

Usage: python tools/eigen_gap.py [--out profiles/r02_eigen_gap.json] [--jobs 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from computervision_objectdetection_featurematching_amd.synthetic import apply_h, random_homography  # noqa: E402
from oracle import oracle as O  # noqa: E402

ULPS = (1, 2, 4, 1 << 12, 1 << 20, 1 << 28)  # < 2^31 (the knob is an int)
SEEDS = (1, 2, 3)


def make_problems(cfg: str):
    rng = np.random.default_rng({"c1": 0xE1, "c2": 0xE2, "c3": 0xE3}[cfg])
    spec = {"c1": (145, 2000), "c2": (40, 2000), "c3": (16, 50000)}[cfg]
    out = []
    for _ in range(spec[0]):
        if cfg == "c1":
            n = int(rng.integers(10, 301))
            w = float(rng.uniform(0.2, 0.8))
        else:
            n = 400 if cfg == "c2" else 2000
            w = 0.08
        src = np.c_[rng.uniform(0, 640, n), rng.uniform(0, 480, n)].astype(np.float32)
        dst = np.c_[rng.uniform(0, 640, n), rng.uniform(0, 480, n)].astype(np.float32)
        k = max(int(round(w * n)), 4)
        inl = rng.choice(n, size=k, replace=False)
        dst[inl] = apply_h(random_homography(rng), src[inl]) + rng.uniform(-0.5, 0.5, (k, 2)).astype(np.float32)
        out.append((src, dst, spec[1]))
    return out


def run_one(args):
    src, dst, max_iters, ulps, seed = args
    O.set_model_perturbation(ulps, seed)
    r, counts = O.ransac_counts(src, dst, max_iters=max_iters)
    ok, H, mask = O.find_homography(src, dst, max_iters=max_iters)
    O.set_model_perturbation(0, 0)
    return dict(rmask=r["mask"].tobytes(), iters=r["iters"], best=r["best_iter"], ok=int(ok),
                H=H.reshape(9).tolist(), mask=mask.tobytes(), counts=counts)


def study(cfg: str, jobs: int):
    probs = make_problems(cfg)
    tasks = [(s, d, mi, 0, 0) for s, d, mi in probs]
    tasks += [(s, d, mi, u, sd) for u in ULPS for sd in SEEDS for s, d, mi in probs]
    t0 = time.time()
    with Pool(jobs) as pool:
        res = pool.map(run_one, tasks, chunksize=1)
    n = len(probs)
    base = res[:n]
    rows = {}
    for a, u in enumerate(ULPS):
        c = dict(runs=0, rmask=0, iters=0, best_iter=0, status=0, final_mask=0, mask_bits_flipped=0,
                 max_rel_dH=0.0, hypotheses=0, hypothesis_counts_changed=0)
        for b, _ in enumerate(SEEDS):
            for i in range(n):
                r = res[n + (a * len(SEEDS) + b) * n + i]
                o = base[i]
                c["runs"] += 1
                c["rmask"] += r["rmask"] != o["rmask"]
                c["iters"] += r["iters"] != o["iters"]
                c["best_iter"] += r["best"] != o["best"]
                c["status"] += r["ok"] != o["ok"]
                c["final_mask"] += r["mask"] != o["mask"]
                k = min(len(r["counts"]), len(o["counts"]))
                c["hypotheses"] += k
                c["hypothesis_counts_changed"] += int(np.sum(r["counts"][:k] != o["counts"][:k]))
                c["mask_bits_flipped"] += int(np.sum(np.frombuffer(r["mask"], np.uint8) != np.frombuffer(o["mask"], np.uint8)))
                if r["ok"] and o["ok"]:
                    h1, h0 = np.array(r["H"]), np.array(o["H"])
                    c["max_rel_dH"] = max(c["max_rel_dH"], float(np.max(np.abs(h1 - h0) / np.maximum(np.abs(h0), 1e-12))))
        rows[f"{u}ulp"] = c
    return dict(config=cfg, problems=n, max_iters=probs[0][2], seconds=round(time.time() - t0, 1),
                accepted_unperturbed=int(sum(b["ok"] for b in base)), per_ulp=rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_eigen_gap.json"))
    ap.add_argument("--jobs", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--configs", default="c1,c2,c3")
    a = ap.parse_args()
    O.build()
    out = [study(c, a.jobs) for c in a.configs.split(",")]
    for s in out:
        print(f"{s['config']}: {s['problems']} problems, maxIters {s['max_iters']}, {s['seconds']} s")
        for k, c in s["per_ulp"].items():
            r = c["runs"]
            print(f"  {k:>5}: runs {r}  ransac-mask {c['rmask']}  iters {c['iters']}  best-iter {c['best_iter']}  "
                  f"status {c['status']}  final-mask {c['final_mask']} ({c['mask_bits_flipped']} bits)  "
                  f"max rel dH {c['max_rel_dH']:.2e}  hypotheses {c['hypotheses']} "
                  f"(count changed {c['hypothesis_counts_changed']})")
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
