"""Host stages after the matcher (include/mim_detect.hpp) against oracle/detect_oracle.py — CPU only.

* boxes: clustering (TestsDetector.cpp:112-151), margins (:160-183), cluster boxes, merge (:193-236),
  area gate (:239-248) on synthetic inlier-point clouds — blobs that chain, blobs that merge, blobs
  below 18 points, scaled points (x / 0.7 ...), duplicates, a NaN point.  Everything bit-exact: the
  clusters in order, every margin's float bits, every box.
* results + metrics end to end on the reference's own label files (tests/golden/dataset, copied from
  /root/reference/data/*/labels): boxes built from points planted around each ground-truth box go
  through boxes_for_model -> save_detections (utils.cpp:12-20 format) -> the metrics
  (metrics.cpp:12-186), C++ against the oracle.
"""
import math
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import detect_oracle as D

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATASET = os.path.join(ROOT, "tests", "golden", "dataset")


def build_driver(exe, sanitize=False):
    """tests/cpp/test_detect.cpp over include/mim_detect.hpp; sanitize: ASan + UBSan, any
    finding aborts the driver, so every test below fails on it."""
    san = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
    subprocess.check_call(["g++", "-std=c++17", *(san if sanitize else ["-O2"]), "-Wall", "-Wextra",
                           os.path.join(ROOT, "tests", "cpp", "test_detect.cpp"), "-o", exe])
    return exe


@pytest.fixture(scope="module", params=["plain", "asan+ubsan"])
def driver(tmp_path_factory, request):
    exe = str(tmp_path_factory.mktemp("detect") / "test_detect")
    return build_driver(exe, sanitize=request.param != "plain")


def _write_points(path, pts, eps=20.0, min_points=18, merge=250.0, min_area=2500, factor=1.0):
    with open(path, "wb") as f:
        f.write(struct.pack("<ififif", len(pts), eps, min_points, merge, min_area, factor))
        f.write(np.asarray(pts, np.float32).reshape(-1, 2).tobytes())


def _parse(path):
    out = dict(order=None, clusters=[], margins=[], cluster_boxes=[], discarded=None, merged=[], rejected=[], dets=[])
    for line in open(path):
        t = line.split()
        if t[0] == "order":
            out["order"] = [int(v) for v in t[2:]]
        elif t[0] in ("cluster", "discarded"):
            vals = [float.fromhex(v) for v in t[2:]]
            pts = [(vals[k], vals[k + 1]) for k in range(0, len(vals), 2)]
            if t[0] == "cluster":
                out["clusters"].append(pts)
            else:
                out["discarded"] = pts
        elif t[0] == "margin":
            out["margins"].append(float.fromhex(t[1]))
        elif t[0] == "clusterbox":
            out["cluster_boxes"].append(tuple(int(v) for v in t[1:]))
        elif t[0] in ("merged", "rejected", "det"):
            out[{"merged": "merged", "rejected": "rejected", "det": "dets"}[t[0]]].append(tuple(int(v) for v in t[1:]))
    return out


def _run_boxes(driver, tmp_path, pts, **kw):
    fin, fout = str(tmp_path / "pts.bin"), str(tmp_path / "out.txt")
    _write_points(fin, pts, **kw)
    subprocess.check_call([driver, "boxes", fin, fout])
    return _parse(fout)


def _same_pts(a, b):
    a = np.asarray(a, np.float32).reshape(-1, 2)
    b = np.asarray(b, np.float32).reshape(-1, 2)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _scene(seed, n_blobs=6, noise=40):
    rng = np.random.default_rng(seed)
    pts = []
    for _ in range(n_blobs):
        c = rng.uniform(50, 1200, 2)
        k = int(rng.integers(5, 120))
        s = rng.uniform(3, 14)
        pts.append(c + rng.normal(scale=s, size=(k, 2)))
        if rng.random() < 0.3:  # a neighbour blob: merged box or a chained cluster
            pts.append(c + rng.uniform(30, 200, 2) + rng.normal(scale=s, size=(int(rng.integers(18, 60)), 2)))
    pts.append(rng.uniform(0, 1280, (noise, 2)))
    p = np.concatenate(pts).astype(np.float32)
    # the reference divides each scale's points by the scale (TestsDetector.cpp:48-55)
    scale = np.float32(rng.choice([0.7, 0.85, 1.0, 1.15, 1.3]))
    p = (p.astype(np.float32) * scale).astype(np.float32) / scale
    p[rng.choice(len(p), 3)] = p[rng.choice(len(p), 3)]  # duplicated points
    return p[rng.permutation(len(p))]


@pytest.mark.parametrize("seed", range(12))
def test_boxes_match_oracle(driver, tmp_path, seed):
    pts = _scene(seed)
    if seed == 3:
        pts = np.vstack([pts, [[np.nan, 5.0]]]).astype(np.float32)
    got = _run_boxes(driver, tmp_path, pts)
    assert sorted(got["order"]) == list(range(len(pts)))
    ref = D.boxes_for_model(pts, got["order"])
    assert len(got["clusters"]) == len(ref["kept"])
    for gc, rc in zip(got["clusters"], ref["kept"]):
        assert _same_pts(gc, pts[rc])
    assert _same_pts(got["discarded"], pts[ref["discarded"]] if ref["discarded"] else np.zeros((0, 2)))
    assert [np.float32(m).tobytes() for m in got["margins"]] == [m.tobytes() for m in ref["margins"]]
    assert got["cluster_boxes"] == ref["cluster_boxes"]
    assert got["merged"] == ref["merged"]
    assert got["rejected"] == ref["rejected"]
    assert got["dets"] == ref["dets"]


def test_boxes_edge_cases(driver, tmp_path):
    # empty input; a single cluster of exactly 18 and one of 17; points exactly 20 apart (link <= eps);
    # a box below the area gate
    assert _run_boxes(driver, tmp_path, np.zeros((0, 2), np.float32))["dets"] == []
    line18 = np.c_[np.arange(18) * 20.0, np.zeros(18)].astype(np.float32)
    line17 = np.c_[np.arange(17) * 20.0, np.full(17, 1000.0)].astype(np.float32)
    got = _run_boxes(driver, tmp_path, np.vstack([line18, line17]))
    ref = D.boxes_for_model(np.vstack([line18, line17]), got["order"])
    assert len(got["clusters"]) == 1 and len(got["clusters"][0]) == 18 and len(got["discarded"]) == 17
    assert got["cluster_boxes"] == ref["cluster_boxes"] and got["dets"] == ref["dets"]
    tight = (np.random.default_rng(1).normal(scale=1.0, size=(30, 2)) + 300).astype(np.float32)
    got = _run_boxes(driver, tmp_path, tight)
    assert got["dets"] == [] and len(got["rejected"]) == 1  # a ~6 px box: area < 2500
    assert got["rejected"] == D.boxes_for_model(tight, got["order"])["rejected"]


def test_boxes_scaled_threshold_params(driver, tmp_path):
    pts = _scene(99, n_blobs=10)
    kw = dict(eps=12.5, min_points=10, merge=120.0, min_area=900, factor=1.5)
    got = _run_boxes(driver, tmp_path, pts, **kw)
    ref = D.boxes_for_model(pts, got["order"], kw["eps"], kw["min_points"], kw["merge"], kw["min_area"], kw["factor"])
    assert got["cluster_boxes"] == ref["cluster_boxes"] and got["merged"] == ref["merged"] and got["dets"] == ref["dets"]


def _gt_boxes():
    return {c: D.read_boxes(os.path.join(DATASET, c, "labels")) for c in sorted(os.listdir(DATASET))}


def test_golden_labels_read():
    gt = _gt_boxes()
    assert set(gt) == {"004_sugar_box", "006_mustard_bottle", "035_power_drill"}
    assert sum(len(v) for v in gt.values()) == 30
    assert gt["004_sugar_box"]["4_0001_000121"]["004_sugar_box"] == [397, 235, 469, 460]


def test_results_and_metrics_end_to_end(driver, tmp_path):
    """Scene points planted inside (shrunken) ground-truth boxes -> boxes_for_model -> results files ->
    mean IoU / per-class IoU / accuracy, C++ (mim_detect.hpp) vs the oracle, on the reference's labels."""
    rng = np.random.default_rng(2024)
    out_cpp, out_py = tmp_path / "out_cpp", tmp_path / "out_py"
    for cls, files in _gt_boxes().items():
        (out_cpp / cls).mkdir(parents=True)
        (out_py / cls).mkdir(parents=True)
        for fid, objs in sorted(files.items()):
            # one results file per scene, "<scene>_results.txt" with scene = "<id>-color" (Output.cpp:44-45);
            # the reference appends each model's detections in model order (TestsDetector.cpp:38, :247)
            scene_cpp, scene_py = [], []
            for oid, (x0, y0, x1, y1) in sorted(objs.items()):
                if rng.random() < 0.15 or (oid != cls and rng.random() < 0.5):
                    continue  # a model that found nothing in this scene
                w, h = x1 - x0, y1 - y0
                k = int(rng.integers(25, 200))
                shrink = rng.uniform(0.05, 0.35)
                pts = np.c_[rng.uniform(x0 + shrink * w, x1 - shrink * w, k),
                            rng.uniform(y0 + shrink * h, y1 - shrink * h, k)].astype(np.float32)
                if rng.random() < 0.3:  # a second part of the object: two clusters, one merged box
                    pts = np.vstack([pts, pts[: k // 2] + np.float32(rng.uniform(-30, 30, 2))])
                fin, fo = str(tmp_path / "p.bin"), str(tmp_path / "o.txt")
                part = str(tmp_path / "part.txt")
                _write_points(fin, pts)
                subprocess.check_call([driver, "boxes", fin, fo, part, oid])
                scene_cpp.append(open(part).read())
                got = _parse(fo)
                ref = D.boxes_for_model(pts, got["order"])
                assert got["dets"] == ref["dets"]
                D.save_detections(part, ref["dets"], oid)
                scene_py.append(open(part).read())
            with open(out_cpp / cls / f"{fid}-color_results.txt", "w") as f:
                f.write("".join(scene_cpp))
            with open(out_py / cls / f"{fid}-color_results.txt", "w") as f:
                f.write("".join(scene_py))
    # byte-identical results files (utils.cpp:12-20 format)
    for cls in os.listdir(out_cpp):
        for fn in os.listdir(out_cpp / cls):
            assert open(out_cpp / cls / fn).read() == open(out_py / cls / fn).read(), fn
    r = subprocess.run([driver, "metrics", DATASET, str(out_cpp)], capture_output=True, text=True, check=True)
    vals = {}
    for line in r.stdout.splitlines():
        t = line.split()
        vals[tuple(t[:-1])] = float.fromhex(t[-1])
    assert np.float32(vals[("mean_iou",)]) == D.mean_iou(DATASET, str(out_py))
    for cls in os.listdir(DATASET):
        assert np.float32(vals[("class_iou", cls)]) == D.class_iou(os.path.join(DATASET, cls, "labels"), str(out_py / cls))
    acc = D.accuracy(DATASET, str(out_py))
    for c, a in acc.items():
        assert np.float32(vals[("accuracy", c)]) == a
    assert 0.1 < vals[("mean_iou",)] < 1.0 and not math.isnan(vals[("mean_iou",)])
