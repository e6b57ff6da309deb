"""CPU restatement of the reference's host stages after the matcher — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module (as the checker of include/mim_detect.hpp).  Each function restates
the reference code it cites with the same arithmetic types (numpy float32 where the reference computes
in float, float64 where it computes in double):

  cluster_points   /root/reference/src/TestsDetector.cpp:112-151
  bounding_rect    cv::boundingRect of CV_32F points (OpenCV imgproc shapedescr.cpp, recalled: corners
                   floored, width = floor(xmax) - floor(xmin) + 1)
  cluster_margin   TestsDetector.cpp:160-183
  cluster_box      TestsDetector.cpp:157-187
  merge_boxes      TestsDetector.cpp:193-236
  boxes_for_model  TestsDetector.cpp:112-248
  read_boxes / iou / mean_iou / class_iou / accuracy    src/metrics.cpp:12-186
  save_detections  src/utils.cpp:12-20

The reference's BFS visits the points in the iteration order of a std::unordered_set<size_t>
(TestsDetector.cpp:114-134), a property of the C++ standard library, not of the algorithm; the
caller passes that order (the test driver prints the libstdc++ order it was built against).  Parity
status: pinned to the reference's own source text and, for the metrics, to its own label files
(tests/golden/dataset); cv::boundingRect's float rule is recalled OpenCV behaviour (OpenCV is absent).
"""
from __future__ import annotations

import math
import os
from collections import deque

import numpy as np

F32 = np.float32


def _dist(a, b) -> np.float32:
    """(float)cv::norm(a - b) for Point2f a, b: float differences, double sqrt, cast to float."""
    dx = F32(F32(a[0]) - F32(b[0]))
    dy = F32(F32(a[1]) - F32(b[1]))
    return F32(math.sqrt(float(dx) * float(dx) + float(dy) * float(dy)))


def cluster_points(pts, order, eps=20.0, min_points=18):
    """TestsDetector.cpp:112-151 with the set's visiting order `order` (a permutation of range(n))."""
    eps = F32(eps)
    unassigned = list(order)  # the set, in iteration order; erasing keeps the rest in order
    kept, discarded = [], []
    while unassigned:
        start = unassigned.pop(0)
        cur = [start]
        todo = deque([start])
        while todo:
            c = todo.popleft()
            take = [o for o in unassigned if _dist(pts[c], pts[o]) <= eps]
            for o in take:
                cur.append(o)
                todo.append(o)
            if take:
                s = set(take)
                unassigned = [o for o in unassigned if o not in s]
        (kept if len(cur) >= min_points else discarded).append(cur)
    return kept, [i for c in discarded for i in c]


def bounding_rect(pts):
    xs = [F32(p[0]) for p in pts]
    ys = [F32(p[1]) for p in pts]
    x0, x1 = math.floor(min(xs)), math.floor(max(xs))
    y0, y1 = math.floor(min(ys)), math.floor(max(ys))
    return (x0, y0, x1 - x0 + 1, y1 - y0 + 1)


def cluster_margin(pts, factor=1.0):
    d = []
    mean = F32(0)
    for i in range(len(pts)):
        for j in range(i + 1, len(pts)):
            v = _dist(pts[i], pts[j])
            d.append(v)
            mean = F32(mean + v)
    if d:
        mean = F32(mean / F32(len(d)))
    var = F32(0)
    for v in d:
        dv = F32(v - mean)
        var = F32(var + F32(float(dv) * float(dv)))
    return F32(F32(np.sqrt(F32(var / F32(len(d))))) * F32(factor))


def cluster_box(pts, factor=1.0):
    x, y, w, h = bounding_rect(pts)
    m = cluster_margin(pts, factor)
    return (x - int(m), y - int(m), w + int(F32(2) * m), h + int(F32(2) * m))


def merge_boxes(boxes, max_dist=250.0):
    def centre(b):
        return (F32(F32(b[0]) + F32(F32(b[2]) / F32(2))), F32(F32(b[1]) + F32(F32(b[3]) / F32(2))))

    done = [False] * len(boxes)
    out = []
    for i in range(len(boxes)):
        if done[i]:
            continue
        done[i] = True
        group = []
        q = deque([i])
        while q:
            c = q.popleft()
            group.append(boxes[c])
            cc = centre(boxes[c])
            for j in range(len(boxes)):
                if done[j]:
                    continue
                cj = centre(boxes[j])
                dx, dy = F32(cc[0] - cj[0]), F32(cc[1] - cj[1])
                if math.sqrt(float(dx) * float(dx) + float(dy) * float(dy)) <= float(F32(max_dist)):
                    done[j] = True
                    q.append(j)
        x0 = min(b[0] for b in group)
        y0 = min(b[1] for b in group)
        x1 = max(b[0] + b[2] for b in group)
        y1 = max(b[1] + b[3] for b in group)
        out.append((x0, y0, x1 - x0, y1 - y0))
    return out


def boxes_for_model(pts, order, eps=20.0, min_points=18, merge=250.0, min_area=2500, factor=1.0):
    """TestsDetector.cpp:112-248: clusters (index lists), discarded indices, cluster boxes, merged,
    rejected and accepted boxes."""
    res = dict(kept=[], discarded=[], margins=[], cluster_boxes=[], merged=[], rejected=[], dets=[])
    if len(pts) == 0:
        return res
    kept, disc = cluster_points(pts, order, eps, min_points)
    res["kept"], res["discarded"] = kept, disc
    if not kept:
        return res
    for c in kept:
        cp = [pts[i] for i in c]
        res["margins"].append(cluster_margin(cp, factor))
        res["cluster_boxes"].append(cluster_box(cp, factor))
    res["merged"] = merge_boxes(res["cluster_boxes"], merge)
    for b in res["merged"]:
        (res["rejected"] if b[2] * b[3] < min_area else res["dets"]).append(b)
    return res


def save_detections(path, dets, name):
    with open(path, "w") as f:
        for x, y, w, h in dets:
            f.write(f"{name} {x} {y} {x + w} {y + h}\n")


def read_boxes(directory):
    """metrics.cpp:56-75"""
    boxes = {}
    for e in os.scandir(directory):
        fid = e.name.split("-", 1)[0]
        with open(e.path) as f:
            tok = f.read().split()
        for k in range(0, len(tok) - 4, 5):
            try:
                boxes.setdefault(fid, {})[tok[k]] = [int(t) for t in tok[k + 1:k + 5]]
            except ValueError:
                break
    return boxes


def iou(p, q):
    """metrics.cpp:88-104 (int areas, float ratio)"""
    iw = max(0, min(p[2], q[2]) - max(p[0], q[0]))
    ih = max(0, min(p[3], q[3]) - max(p[1], q[1]))
    inter = iw * ih
    uni = (p[2] - p[0]) * (p[3] - p[1]) + (q[2] - q[0]) * (q[3] - q[1]) - inter
    return F32(F32(inter) / F32(uni))


def class_iou(gt_dir, pred_dir):
    """metrics.cpp:29-53"""
    gt, pred = read_boxes(gt_dir), read_boxes(pred_dir)
    total, count = F32(0), 0
    for fid in sorted(gt):
        for oid in sorted(gt[fid]):
            p = pred.get(fid, {})
            v = iou(gt[fid][oid], p[oid]) if oid in p else F32(0)
            count += 1
            if v > 0:
                total = F32(total + v)
    return F32(total / F32(count)) if count else F32(0)


def mean_iou(dataset, output, gt_sub="labels"):
    """metrics.cpp:12-26 (class directories in directory order)"""
    per = [class_iou(os.path.join(e.path, gt_sub), os.path.join(output, e.name))
           for e in os.scandir(dataset) if e.is_dir()]
    if not per:
        return F32(0)
    s = F32(0)
    for v in per:
        s = F32(s + v)
    return F32(s / F32(len(per)))


def accuracy(dataset, output, gt_sub="labels"):
    """metrics.cpp:107-186"""
    total, tp = {}, {}
    for e in os.scandir(dataset):
        if not e.is_dir():
            continue
        gt = read_boxes(os.path.join(e.path, gt_sub))
        pred = read_boxes(os.path.join(output, e.name))
        for fid, objs in gt.items():
            for oid, box in objs.items():
                cls = oid.split("_", 1)[0]
                total[cls] = total.get(cls, 0) + 1
                if oid in pred.get(fid, {}) and iou(box, pred[fid][oid]) >= F32(0.5):
                    tp[cls] = tp.get(cls, 0) + 1
    return {c: (F32(F32(tp.get(c, 0)) / F32(n)) if n else F32(0)) for c, n in total.items()}
