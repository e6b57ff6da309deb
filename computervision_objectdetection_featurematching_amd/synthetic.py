"""Seeded synthetic SIFT-like workloads for the matcher + RANSAC hot path.

SURVEY.md §8(d) "Synthetic inputs": the reference's only data are images that need OpenCV SIFT to
become descriptors (src/ModelsDetector.cpp:75, src/TestsDetector.cpp:106), which nothing in this
image can run, so the benches and tests use descriptors drawn in SIFT's value domain:

* 128 gamma(0.5) values, L2-normalised, clipped at 0.2, renormalised, x512, rounded, saturated to
  [0, 255] and stored as float32 — the integer-valued CV_32F rows OpenCV SIFT emits
  (SURVEY.md Appendix A.3), so squared distances are exact integers < 2^24.
* A scene ("train" side, the scaled scene descriptors of TestsDetector.cpp:106) holds, for every
  model, ``n_plant`` noisy copies (+-1..2 on <= 8 dims) of that model's first ``n_plant`` rows at
  random positions; the remaining rows are fresh random descriptors.
* Keypoints are uniform in [0,640)x[0,480).  For a fraction ``inlier_frac`` of each model's planted
  rows the scene keypoint is H_true(model keypoint) + U(+-0.5 px); the rest are random.  H_true is a
  random mild perspective (|h6|,|h7| ~ 1e-4), one per (model, scene).

Problem (m, s) = knnMatch(model m, scene s) + ratio + findHomography (TestsDetector.cpp:58-95).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

DIM = 128
IMG_W, IMG_H = 640.0, 480.0
SEED_BASE = 0x5EED0000


def sift_like(rng: np.random.Generator, n: int, dim: int = DIM) -> np.ndarray:
    v = rng.gamma(0.5, 1.0, size=(n, dim)).astype(np.float64)
    v /= np.maximum(np.linalg.norm(v, axis=1, keepdims=True), 1e-12)
    v = np.minimum(v, 0.2)
    v *= 512.0 / np.maximum(np.linalg.norm(v, axis=1, keepdims=True), 1e-12)
    return np.clip(np.rint(v), 0, 255).astype(np.float32)


def perturb(rng: np.random.Generator, d: np.ndarray) -> np.ndarray:
    out = d.copy()
    n = out.shape[0]
    k = rng.integers(1, 9, size=n)
    for i in range(n):
        cols = rng.choice(out.shape[1], size=k[i], replace=False)
        delta = rng.choice(np.array([-2, -1, 1, 2], dtype=np.float32), size=k[i])
        out[i, cols] = np.clip(out[i, cols] + delta, 0, 255)
    return out


def random_homography(rng: np.random.Generator) -> np.ndarray:
    ang = rng.uniform(-0.25, 0.25)
    sc = rng.uniform(0.8, 1.25)
    c, s = np.cos(ang) * sc, np.sin(ang) * sc
    H = np.array([[c, -s, rng.uniform(-40, 40)],
                  [s, c, rng.uniform(-40, 40)],
                  [rng.uniform(-1e-4, 1e-4), rng.uniform(-1e-4, 1e-4), 1.0]])
    return H


def apply_h(H: np.ndarray, xy: np.ndarray) -> np.ndarray:
    p = np.c_[xy.astype(np.float64), np.ones(len(xy))] @ H.T
    return (p[:, :2] / p[:, 2:3]).astype(np.float32)


@dataclass
class Dataset:
    model_desc: list      # n_models x (nq, 128) float32
    model_kp: list        # n_models x (nq, 2) float32
    scene_desc: list      # n_scenes x (nt, 128) float32
    scene_kp: list        # n_scenes x (nt, 2) float32
    H_true: np.ndarray    # (n_models, n_scenes, 3, 3)
    plant_pos: np.ndarray  # (n_models, n_scenes, n_plant) train row of each planted copy
    n_plant: int
    n_inl: int

    @property
    def problems(self):
        return [(m, s) for m in range(len(self.model_desc)) for s in range(len(self.scene_desc))]


def make_dataset(n_models: int, n_scenes: int, nq: int, nt: int, n_plant: int,
                 inlier_frac: float = 0.08, seed: int = SEED_BASE, scene_ids=None) -> Dataset:
    """``scene_ids``: generate only these scenes of the ``n_scenes``-scene batch (scene s is seeded by
    ``seed + 1 + s`` alone, so a rank's shard of a global batch is the same data whichever rank, and
    however many ranks, generate it: C4's sharding, bench.py)."""
    if n_models * n_plant > nt or n_plant > nq:
        raise ValueError("planted rows do not fit")
    ids = list(range(n_scenes)) if scene_ids is None else [int(x) for x in scene_ids]
    mrng = np.random.default_rng(seed)
    model_desc, model_kp = [], []
    for _ in range(n_models):
        model_desc.append(sift_like(mrng, nq))
        model_kp.append(np.c_[mrng.uniform(0, IMG_W, nq), mrng.uniform(0, IMG_H, nq)].astype(np.float32))
    n_inl = int(round(inlier_frac * n_plant))
    scene_desc, scene_kp = [], []
    H_true = np.zeros((n_models, len(ids), 3, 3))
    plant_pos = np.zeros((n_models, len(ids), n_plant), dtype=np.int64)
    for s, gs in enumerate(ids):
        srng = np.random.default_rng(seed + 1 + gs)
        d = sift_like(srng, nt)
        kp = np.c_[srng.uniform(0, IMG_W, nt), srng.uniform(0, IMG_H, nt)].astype(np.float32)
        pos = srng.permutation(nt)[: n_models * n_plant].reshape(n_models, n_plant)
        for m in range(n_models):
            d[pos[m]] = perturb(srng, model_desc[m][:n_plant])
            H = random_homography(srng)
            H_true[m, s] = H
            inl = srng.choice(n_plant, size=n_inl, replace=False)
            proj = apply_h(H, model_kp[m][inl])
            kp[pos[m][inl]] = proj + srng.uniform(-0.5, 0.5, size=proj.shape).astype(np.float32)
            plant_pos[m, s] = pos[m]
        scene_desc.append(d)
        scene_kp.append(kp)
    return Dataset(model_desc, model_kp, scene_desc, scene_kp, H_true, plant_pos, n_plant, n_inl)


def make_ragged_dataset(nqs, nts, scene_plant_frac: float = 0.5, inlier_frac: float = 0.5,
                        seed: int = SEED_BASE) -> Dataset:
    """Ragged problem shapes of the reference's own run (SURVEY.md §8(d) C1 surrogate): model views of
    ``nqs[v]`` rows (an ObjectModel's masked SIFT views, ~100-500 keypoints) against scaled scenes of
    ``nts[s]`` rows (~1k-4k).  A fraction ``scene_plant_frac`` of every scene's rows are noisy copies
    of view rows, split evenly over the views (``n_plant[v, s]`` rows of view v), of which
    ``inlier_frac`` sit at H_true(v, s) of the view keypoint: every problem has a few to a few dozen
    good matches and stops early or runs its 2000 iterations, as real detections do."""
    nv, ns = len(nqs), len(nts)
    mrng = np.random.default_rng(seed)
    model_desc = [sift_like(mrng, int(n)) for n in nqs]
    model_kp = [np.c_[mrng.uniform(0, IMG_W, int(n)), mrng.uniform(0, IMG_H, int(n))].astype(np.float32)
                for n in nqs]
    n_plant = np.zeros((nv, ns), np.int64)
    H_true = np.zeros((nv, ns, 3, 3))
    plant_pos = np.full((nv, ns, max(int(n) for n in nqs)), -1, np.int64)
    scene_desc, scene_kp = [], []
    for s in range(ns):
        nt = int(nts[s])
        srng = np.random.default_rng(seed + 1 + s)
        d = sift_like(srng, nt)
        kp = np.c_[srng.uniform(0, IMG_W, nt), srng.uniform(0, IMG_H, nt)].astype(np.float32)
        per_view = int(scene_plant_frac * nt) // nv
        free = srng.permutation(nt)
        used = 0
        for v in range(nv):
            k = min(per_view, int(nqs[v]))
            rows = srng.choice(int(nqs[v]), size=k, replace=False)
            pos = free[used:used + k]
            used += k
            d[pos] = perturb(srng, model_desc[v][rows])
            H = random_homography(srng)
            H_true[v, s] = H
            ninl = int(round(inlier_frac * k))
            inl = srng.choice(k, size=ninl, replace=False)
            proj = apply_h(H, model_kp[v][rows[inl]])
            kp[pos[inl]] = proj + srng.uniform(-0.5, 0.5, size=proj.shape).astype(np.float32)
            n_plant[v, s] = k
            plant_pos[v, s, :k] = pos
        scene_desc.append(d)
        scene_kp.append(kp)
    return Dataset(model_desc, model_kp, scene_desc, scene_kp, H_true, plant_pos, n_plant, -1)


def c1_shapes(seed: int = SEED_BASE):
    """C1 surrogate shapes: sugar_box's 29 model views x the 5 scales of one scene
    (TestsDetector.cpp:58,99) = 145 problems, Nq in [100, 500], Nt in [1000, 4000]."""
    rng = np.random.default_rng(seed ^ 0xC1)
    nqs = rng.integers(100, 501, size=29)
    nts = np.sort(rng.integers(1000, 4001, size=5))  # scales 0.7 .. 1.3: more keypoints when larger
    return nqs, nts


def make_config_dataset(name: str, seed: int = SEED_BASE, scene_ids=None) -> Dataset:
    cfg = CONFIGS[name]
    if cfg.get("ragged"):
        nqs, nts = c1_shapes(seed)
        return make_ragged_dataset(nqs, nts, seed=seed)
    return make_dataset(cfg["n_models"], cfg["n_scenes"], cfg["nq"], cfg["nt"], cfg["n_plant"], seed=seed,
                        scene_ids=scene_ids)


# Configs of BASELINE.json: C1 is the reference's own real-data case (no SIFT here: its surrogate
# shapes); C4 is one global 256-scene batch (1 model set) whose scenes are sharded
# over the GPUs; C5 is the distance kernel alone.
CONFIGS = {
    "c1": dict(ragged=True, n_models=29, n_scenes=5, nq=500, nt=4000, max_iters=2000),
    "c2": dict(n_models=1, n_scenes=1, nq=2000, nt=2000, n_plant=400, max_iters=2000),
    "c3": dict(n_models=3, n_scenes=32, nq=10000, nt=10000, n_plant=2000, max_iters=50000),
    "c4": dict(n_models=1, n_scenes=256, nq=10000, nt=10000, n_plant=2000, max_iters=50000, sharded=True),
    "c5": dict(n_models=1, n_scenes=1, nq=50000, nt=50000, n_plant=0, max_iters=0, knn_only=True),
}
