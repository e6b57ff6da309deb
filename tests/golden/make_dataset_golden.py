"""The reference's whole run (main.cpp:17-33) on its own data, by the CPU restatement: every object's
models against every test image, results files and the metrics — the golden of
tests/test_dataset_gpu.py.

Run HERE (needs /root/reference; ~15 min on 8 cores):  python tests/golden/make_dataset_golden.py
Writes
  tests/golden/dataset_gray.npz   <obj>/view/<name>, <obj>/mask/<name> (ModelsDetector.cpp:51,61) and
                                   <obj>/scene/<id> (Output.cpp:34 + preprocessing.cpp:11) for the 3 objects:
                                   gray by cvtColor's fixed-point formula (see make_sift_fixtures.py)
  tests/golden/dataset_expected.json  per scene ("<obj>/<id>"): the detections [[x, y, w, h, name], ...]
                                   of detectObjects against all models, in model order, plus per model
                                   the number of allUnfilteredScenePts; and the metrics of the results
                                   files (mean IoU, per-class IoU, accuracy) against the label files
Order choices (the reference's are filesystem-dependent): objects (= models) and views sorted by name.
The boxes come from include/mim_detect.hpp through tests/cpp/test_detect.cpp and are checked here
against oracle/detect_oracle.py on the same visiting order; the metrics likewise.
"""
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import detect_oracle as D  # noqa: E402
from oracle import oracle as O  # noqa: E402

REF = "/root/reference/data"
SCALES = (0.7, 0.85, 1.0, 1.15, 1.3)


def to_gray(rgb):
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def load():
    out, objs = {}, sorted(os.listdir(REF))
    for obj in objs:
        mdir = os.path.join(REF, obj, "models")
        for f in sorted(os.listdir(mdir)):
            if f.endswith("_color.png"):
                out[f"{obj}/view/{f[:-10]}"] = to_gray(np.asarray(Image.open(os.path.join(mdir, f)).convert("RGB")))
            elif f.endswith("_mask.png"):
                out[f"{obj}/mask/{f[:-9]}"] = np.asarray(Image.open(os.path.join(mdir, f)).convert("L"))
        tdir = os.path.join(REF, obj, "test_images")
        for f in sorted(os.listdir(tdir)):
            out[f"{obj}/scene/{f[:-10]}"] = to_gray(np.asarray(Image.open(os.path.join(tdir, f)).convert("RGB")))
    return out, objs


def boxes(drv, tmp, P):
    fin, fo = os.path.join(tmp, "p.bin"), os.path.join(tmp, "o.txt")
    with open(fin, "wb") as f:
        f.write(struct.pack("<ififif", len(P), 20.0, 18, 250.0, 2500, 1.0))
        f.write(np.asarray(P, np.float32).tobytes())
    subprocess.check_call([drv, "boxes", fin, fo])
    order, dets = None, []
    for line in open(fo):
        t = line.split()
        if t[0] == "order":
            order = [int(v) for v in t[2:]]
        elif t[0] == "det":
            dets.append(tuple(int(v) for v in t[1:]))
    if len(P):
        assert D.boxes_for_model(P, order)["dets"] == dets, "mim_detect.hpp disagrees with detect_oracle.py"
    return dets


def main():
    imgs, objs = load()
    np.savez_compressed(os.path.join(HERE, "dataset_gray.npz"), **imgs)
    models = []  # (name, [(kp_xy, desc)])
    for obj in objs:
        views = []
        for key in sorted(k for k in imgs if k.startswith(f"{obj}/view/")):
            k, d = O.sift_detect_compute(imgs[key], imgs.get(key.replace("/view/", "/mask/")))
            views.append((np.stack([k["x"], k["y"]], 1).astype(np.float32), d))
        models.append((obj, views))
        print("model", obj, len(views), flush=True)
    tmp = tempfile.mkdtemp()
    drv = os.path.join(tmp, "test_detect")
    subprocess.check_call(["g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "test_detect.cpp"), "-o", drv])
    expected = {"scenes": {}}
    out_dir = os.path.join(tmp, "output")
    for obj in objs:
        os.makedirs(os.path.join(out_dir, obj))
        for key in sorted(k for k in imgs if k.startswith(f"{obj}/scene/")):
            sid = key.split("/")[-1]
            scaled = []
            for s in SCALES:
                sk, sd = O.sift_detect_compute(O.resize_linear_u8(imgs[key], fx=s))
                scaled.append((np.stack([sk["x"], sk["y"]], 1).astype(np.float32), sd, np.float32(s)))
            dets, npts = [], []
            for name, views in models:  # TestsDetector.cpp:38, model order
                pts = []
                for sxy, sd, s in scaled:  # :100
                    for vxy, vd in views:  # :58
                        r = O.match_problem(vd, vxy, sd, sxy, threads=8)
                        if r["status"] == 0:
                            p = sxy[r["good_t"][r["mask"].astype(bool)]]
                            pts.append(p / s if s != np.float32(1.0) else p)
                P = np.concatenate(pts).astype(np.float32) if pts else np.zeros((0, 2), np.float32)
                npts.append(int(len(P)))
                dets += [[*b, name] for b in boxes(drv, tmp, P)]
            expected["scenes"][f"{obj}/{sid}"] = {"detections": dets, "n_points": npts}
            with open(os.path.join(out_dir, obj, f"{sid}-color_results.txt"), "w") as f:  # utils.cpp:12-20
                for x, y, w, h, name in dets:
                    f.write(f"{name} {x} {y} {x + w} {y + h}\n")
            print(obj, sid, dets, npts, flush=True)
    # metrics of the results files against the reference's labels (metrics.cpp)
    labels = os.path.join(HERE, "dataset")
    r = subprocess.run([drv, "metrics", labels, out_dir], capture_output=True, text=True, check=True)
    vals = {}
    for line in r.stdout.splitlines():
        t = line.split()
        vals[" ".join(t[:-1])] = float.fromhex(t[-1])
    assert np.float32(vals["mean_iou"]) == D.mean_iou(labels, out_dir)
    expected["metrics"] = vals
    with open(os.path.join(HERE, "dataset_expected.json"), "w") as f:
        json.dump(expected, f, indent=1)
    print(json.dumps(vals))


if __name__ == "__main__":
    main()
