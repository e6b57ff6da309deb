"""BASELINE.json configs[0] on the reference's own data: the sugar_box model (its 29 views with masks)
against its test views — images plus the expected outputs of the whole detectObjects pipeline.

Run HERE (needs /root/reference):  python tests/golden/make_c1_golden.py
Writes tests/golden/c1_sugar_box.npz:
  view/<name>, mask/<name>   the 29 model views (ModelsDetector.cpp:51,61), names sorted
  scene/<id>                 the 10 test views (Output.cpp:34 + preprocessing.cpp:11)
  (gray conversion: cvtColor BGR2GRAY's fixed-point formula, see make_sift_fixtures.py)
and, for the first N_EXPECTED scenes, the outputs of the CPU restatement (oracle/):
  exp/sift/view/<name>        sha256 of the oracle's keypoints + descriptors of each view
  exp/sift/<id>/<scale>       the same for each scaled scene (resize + detectAndCompute)
  exp/res/<id>                per problem (scale-major, then view): n_good, n_inl, status, iters
  exp/H/<id>                  per problem: H (float64, 9)
  exp/pts/<id>                allUnfilteredScenePts of the model (float32, n x 2)
  exp/boxes/<id>              detections (x, y, w, h): mim_detect.hpp through tests/cpp/test_detect.cpp,
                              checked here against oracle/detect_oracle.py on the same visiting order
The view order is the sorted file order (the reference's unordered_map order depends on the directory
order, ModelsDetector.cpp:29-45).
"""
import hashlib
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

REF = "/root/reference/data/004_sugar_box"
SCALES = (0.7, 0.85, 1.0, 1.15, 1.3)
N_EXPECTED = 3


def to_gray(rgb):
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def sift_hash(k, d):
    return np.frombuffer(hashlib.sha256(k.tobytes() + np.ascontiguousarray(d, np.float32).tobytes()).digest(), np.uint8)


def main():
    out = {}
    names = sorted(f[:-len("_color.png")] for f in os.listdir(os.path.join(REF, "models")) if f.endswith("_color.png"))
    views = []
    for n in names:
        g = to_gray(np.asarray(Image.open(os.path.join(REF, "models", n + "_color.png")).convert("RGB")))
        m = np.asarray(Image.open(os.path.join(REF, "models", n + "_mask.png")).convert("L"))
        out[f"view/{n}"], out[f"mask/{n}"] = g, m
        views.append((n, g, m))
    scenes = sorted(f[:-len("-color.jpg")] for f in os.listdir(os.path.join(REF, "test_images")))
    for s in scenes:
        out[f"scene/{s}"] = to_gray(np.asarray(Image.open(os.path.join(REF, "test_images", s + "-color.jpg")).convert("RGB")))

    vk = []
    for n, g, m in views:
        k, d = O.sift_detect_compute(g, m)
        out[f"exp/sift/view/{n}"] = sift_hash(k, d)
        vk.append((k, d))
    tmp = tempfile.mkdtemp()
    drv = os.path.join(tmp, "test_detect")
    subprocess.check_call(["g++", "-std=c++17", "-O2", os.path.join(ROOT, "tests", "cpp", "test_detect.cpp"), "-o", drv])
    for sid in scenes[:N_EXPECTED]:
        res, Hs, pts = [], [], []
        for s in SCALES:
            scaled = O.resize_linear_u8(out[f"scene/{sid}"], fx=s)
            sk, sd = O.sift_detect_compute(scaled)
            out[f"exp/sift/{sid}/{s}"] = sift_hash(sk, sd)
            sxy = np.stack([sk["x"], sk["y"]], 1)
            for k, d in vk:
                r = O.match_problem(d, np.stack([k["x"], k["y"]], 1), sd, sxy, threads=8)
                res.append((r["n_good"], r["n_inl"], r["status"], r["iters"]))
                Hs.append(r["H"].reshape(9))
                if r["status"] == 0:
                    p = sxy[r["good_t"][r["mask"].astype(bool)]].astype(np.float32)
                    if np.float32(s) != np.float32(1.0):
                        p = p / np.float32(s)
                    pts.append(p)
            print(sid, s, len(sk), flush=True)
        P = np.concatenate(pts).astype(np.float32) if pts else np.zeros((0, 2), np.float32)
        fin, fo = os.path.join(tmp, "p.bin"), os.path.join(tmp, "o.txt")
        with open(fin, "wb") as f:
            f.write(struct.pack("<ififif", len(P), 20.0, 18, 250.0, 2500, 1.0))
            f.write(P.tobytes())
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
        out[f"exp/res/{sid}"] = np.array(res, np.int32)
        out[f"exp/H/{sid}"] = np.array(Hs, np.float64)
        out[f"exp/pts/{sid}"] = P
        out[f"exp/boxes/{sid}"] = np.array(dets, np.int32).reshape(-1, 4)
        print(sid, "accepted", int((np.array(res)[:, 2] == 0).sum()), "points", len(P), "boxes", dets, flush=True)
    path = os.path.join(HERE, "c1_sugar_box.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
