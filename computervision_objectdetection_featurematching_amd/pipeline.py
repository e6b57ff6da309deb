"""The reference's detection pipeline on libmim, OpenCV-free: models, detectObjects, results, metrics.

Mirrors (names, argument meaning, outputs):
  ObjectModel                       include/objectModel.hpp:11-16  (name, images, keypoints, descriptors)
  process_model_views               ModelsDetector.cpp:46-80  one object: detectAndCompute(view, mask) per view
  detect_objects                    TestsDetector.cpp:32-251  scene -> [(Rect, model name)]
  save_detections                   utils.cpp:12-20
  process_all_test_images           Output.cpp:15-57          every scene -> results files
Every compute stage runs in libmim: resize and SIFT on the GPU (mim_resize_linear_u8,
mim_sift_detect_compute), the (model, scale, view) problems as ONE device batch (knnMatch k=2 + ratio
+ findHomography RANSAC + gates, mim_batch_run), the boxes in the library's host stage
(mim_detect_boxes = include/mim_detect.hpp).  Images are CV_8UC1 arrays: the grayscale conversion of
preprocessImage (preprocessing.cpp:11) is the caller's (cv::imread(..., IMREAD_GRAYSCALE) or
cvtColor), as is file decoding.

Differences from the reference, all without effect on the result:
  - the scene is resized and SIFT-described once per scale, not once per (model, scale)
    (TestsDetector.cpp:99-107 inside the model loop recomputes the same keypoints per model);
  - view order: the reference iterates an unordered_map filled in directory order
    (ModelsDetector.cpp:29-45), which is filesystem-dependent; here the caller's order is used (the
    clustering's float sums depend on point order, so compare runs with the same view order).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import BoxParams, Rect
from .matcher import DIM, Matcher, default_params

SCALES = (0.7, 0.85, 1.0, 1.15, 1.3)  # TestsDetector.cpp:99


@dataclass
class ObjectModel:  # objectModel.hpp:11-16
    name: str
    images: list = field(default_factory=list)
    keypoints: list = field(default_factory=list)    # KEYPOINT_DTYPE arrays
    descriptors: list = field(default_factory=list)  # (n, 128) float32


def default_box_params(**kw) -> BoxParams:
    p = BoxParams()
    _lib.load().mim_default_box_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def process_model_views(matcher: Matcher, name: str, views) -> ObjectModel:
    """ModelsDetector.cpp:46-80 for one object: views = [(gray, mask or None), ...]."""
    m = ObjectModel(name)
    for gray, mask in views:
        k, d = matcher.sift_detect_compute(gray, mask)
        m.images.append(gray)
        m.keypoints.append(k)
        m.descriptors.append(d)
    return m


def detect_boxes(points: np.ndarray, bp: BoxParams | None = None) -> list[tuple[int, int, int, int]]:
    """TestsDetector.cpp:111-248 for one model's allUnfilteredScenePts -> [(x, y, w, h)]."""
    L = _lib.load()
    pts = np.ascontiguousarray(points, np.float32).reshape(-1, 2)
    bp = bp or default_box_params()
    cap = max(1, len(pts))  # every box holds at least one point: never more boxes than points
    out = (Rect * cap)()
    n = C.c_int32()
    st = L.mim_detect_boxes(C.c_void_p(pts.ctypes.data), len(pts), C.byref(bp), out, cap, C.byref(n))
    if st != 0:
        raise _lib.MimError(st, "mim_detect_boxes failed")
    if n.value > cap:
        raise _lib.MimError(2, f"mim_detect_boxes: {n.value} boxes for {len(pts)} points")
    return [(out[i].x, out[i].y, out[i].width, out[i].height) for i in range(n.value)]


def _model_sets(matcher: Matcher, models: list[ObjectModel]) -> list[list[int]]:
    """The models' views as the matcher's first sets, registered once and kept across scenes: the
    matcher's sets are detect_objects' own; a later call with the same view arrays (by identity) drops
    only the previous scene's sets (mim_sets_truncate), anything else re-registers from scratch."""
    arrays = [d for m in models for d in m.descriptors]
    c = getattr(matcher, "_pipeline_models", None)
    if (c is not None and c["gen"] == matcher.sets_generation and len(c["arrays"]) == len(arrays)
            and all(a is b for a, b in zip(c["arrays"], arrays)) and matcher.n_sets >= c["n"]):
        matcher.truncate_sets(c["n"])
        c["gen"] = matcher.sets_generation
        return c["ids"]
    matcher.clear_sets()
    ids = [[matcher.add_set(d, np.stack([k["x"], k["y"]], 1)) for k, d in zip(m.keypoints, m.descriptors)]
           for m in models]
    matcher._pipeline_models = {"arrays": arrays, "ids": ids, "n": matcher.n_sets, "gen": matcher.sets_generation}
    return ids


def forget_models(matcher: Matcher) -> None:
    """Drop the registered-models cache of _model_sets: call it after rewriting a model's view arrays in
    place (the cache recognises the views by array identity), so the next detect_objects registers them
    anew (mim.hpp's Detector::invalidate_models)."""
    matcher._pipeline_models = None


@dataclass
class SceneRun:
    """detect_objects' intermediate products (for tests and benches)."""
    scene_kp: list      # per scale: KEYPOINT_DTYPE
    scene_desc: list | None  # per scale: (n, 128) float32 copied out of the device sets the batch
    #                          used; None unless detect_objects(..., keep_descriptors=True)
    results: np.ndarray  # RESULT_DTYPE per problem, problems in (model, scale, view) order
    points: list        # per model: allUnfilteredScenePts (n, 2) float32
    detections: list    # [((x, y, w, h), name)]

    def descriptors(self) -> list:
        """scene_desc, or ValueError when the run did not keep them."""
        if self.scene_desc is None:
            raise ValueError("SceneRun.descriptors: detect_objects(..., keep=True) ran without "
                             "keep_descriptors=True (the scene's descriptors stay on the device)")
        return self.scene_desc


def detect_objects(matcher: Matcher, scene_gray, models: list[ObjectModel], scales=SCALES, params=None,
                   box_params: BoxParams | None = None, keep: bool = False, keep_descriptors: bool = False,
                   stage_ms: dict | None = None):
    """detectObjects(scene, models, detector) (TestsDetector.cpp:32-251) on a grayscale scene.

    Returns [((x, y, w, h), name)], or the SceneRun when keep=True (its scene_desc only with
    keep_descriptors: the scene's descriptors never leave the device on the detection path; for the
    caller they are copied out of the very sets the batch matched against, mim_set_rows).
    stage_ms (diagnostic): host wall time of each stage added to it (ms): "sift" (resize + SIFT of every
    scale, sets registered), "match" (the batch enqueued and its records), "gather" (inlier points),
    "boxes"; each stage waits for the device work it needs, so together they are the call's latency."""
    import time as _time
    t_last = [_time.perf_counter()]

    def _mark(name):
        if stage_ms is not None:
            t = _time.perf_counter()
            stage_ms[name] = stage_ms.get(name, 0.0) + 1e3 * (t - t_last[0])
            t_last[0] = t

    params = params or default_params()
    view_ids = _model_sets(matcher, models)
    # :99-107, all scales in one call, the scene's descriptors registered as sets on the device
    scene_ids, _, scene_kp = matcher.sift_scales_to_sets(scene_gray, scales, keypoints=keep)
    scene_desc = [matcher.set_rows(i)[0] for i in scene_ids] if keep_descriptors else None
    _mark("sift")
    # problems in (model, scale, view) order, built as arrays (145 per c1img scene)
    ns = len(scales)
    sid = np.asarray(scene_ids, np.int32)
    probs = np.concatenate([np.stack([np.tile(np.asarray(view_ids[mi], np.int32), ns),
                                      np.repeat(sid, len(view_ids[mi]))], axis=1)
                            for mi in range(len(models))]) if models else np.zeros((0, 2), np.int32)
    prob_scale = np.concatenate([np.repeat(np.asarray(scales, np.float32), len(view_ids[mi]))
                                 for mi in range(len(models))]) if models else np.zeros(0, np.float32)
    res = matcher.match_batch(probs, params)
    _mark("match")
    # :87-94 inlier scene points of the accepted problems (:74, :79, :81, :84), /scale when scale != 1,
    # gathered on the device in batch order; a model's problems are contiguous (model-major order)
    offs, allpts = matcher.batch_inlier_points(len(probs), prob_scale)
    points, i0 = [], 0
    for mi in range(len(models)):
        i1 = i0 + len(scales) * len(view_ids[mi])
        points.append(allpts[offs[i0]:offs[i1]].copy())
        i0 = i1
    _mark("gather")
    dets = []
    for mi, m in enumerate(models):  # :111-248, model order
        dets += [(b, m.name) for b in detect_boxes(points[mi], box_params)]
    _mark("boxes")
    if keep:
        return SceneRun(scene_kp, scene_desc, res, points, dets)
    return dets


def save_detections(path: str, detections) -> None:
    """utils.cpp:12-20: one "<name> x0 y0 x1 y1" line per detection."""
    with open(path, "w") as f:
        for (x, y, w, h), name in detections:
            f.write(f"{name} {x} {y} {x + w} {y + h}\n")


def process_all_test_images(matcher, scenes, models, output_dir: str, params=None,
                            box_params: BoxParams | None = None, rank: int = 0, world: int = 1) -> dict:
    """Output.cpp:15-57 without the file decoding and drawing: scenes = [(object folder, scene name,
    gray image)]; writes <output_dir>/<folder>/<scene name>_results.txt (scene name = the image stem,
    e.g. "4_0001_000121-color") and returns {(folder, scene name): detections}.

    Scenes in flight: `matcher` may be a list of Matchers (library contexts); scene i then runs on
    context i mod len, one host thread per context, so a scene's host stages overlap the other
    contexts' GPU work.  The models are host arrays, registered in each context on its first scene.
    Per-scene results are those of the one-context run (the contexts share no device state), and the
    files and returned dict are the same.

    Several GPUs (one process per GPU, `world` ranks): rank r processes the scenes
    shard.shard_round_robin(len(scenes), world, r) — round robin, since a scene's cost depends on how
    early its problems terminate — and writes their results files; the detections are then
    all-gathered (torch.distributed, the process group the caller created), so every rank returns
    the whole dict, in scene order, and the union of the ranks' files is the one-GPU run's."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    from . import shard
    if isinstance(matcher, Matcher):
        matcher = [matcher]
    if len(matcher) > 1:  # the contexts overlap each other: one stream each (no sampler stream)
        for mm in matcher:
            mm.set_sampler_stream(False)
    mine = list(shard.shard_round_robin(len(scenes), world, rank))
    for i in mine:
        os.makedirs(os.path.join(output_dir, scenes[i][0]), exist_ok=True)
    dets = {}

    def worker(k):
        for j in range(k, len(mine), len(matcher)):
            i = mine[j]
            dets[i] = detect_objects(matcher[k], scenes[i][2], models, params=params, box_params=box_params)

    if len(matcher) == 1:
        worker(0)
    else:
        with ThreadPoolExecutor(len(matcher)) as pool:
            list(pool.map(worker, range(len(matcher))))
    for i in mine:
        folder, name, _ = scenes[i]
        save_detections(os.path.join(output_dir, folder, f"{name}_results.txt"), dets[i])
    parts = shard.gather_objects([(i, dets[i]) for i in mine], world) if world > 1 else [[(i, dets[i]) for i in mine]]
    all_dets = shard.merge_scene_results(parts, len(scenes))
    return {(folder, name): d for (folder, name, _), d in zip(scenes, all_dets)}


__all__ = ["ObjectModel", "SCALES", "SceneRun", "default_box_params", "detect_boxes", "detect_objects",
           "forget_models", "process_all_test_images", "process_model_views", "save_detections", "DIM"]
