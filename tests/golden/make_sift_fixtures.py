"""Grayscale image fixtures for the SIFT / resize parity tests (tests/test_sift_gpu.py).

Run HERE (needs /root/reference, which the GPU box does not have):  python tests/golden/make_sift_fixtures.py
Writes tests/golden/sift_images.npz: a few of the reference's own data files, decoded with PIL and
converted to gray the way the reference does it:
  - model views (ModelsDetector.cpp:51,61): imread(color.png, IMREAD_GRAYSCALE) + imread(mask.png,
    IMREAD_GRAYSCALE).  PNG is lossless; the gray conversion is cvtColor(BGR2GRAY)'s fixed-point
    formula (R*4899 + G*9617 + B*1868 + 2^13) >> 14.  OpenCV's PNG reader lets libpng convert instead,
    which may differ by one level on some pixels: the fixture is an input, not an expected output.
  - scenes (Output.cpp:34 imread IMREAD_COLOR, preprocessing.cpp:11 cvtColor BGR2GRAY): JPEG decoded
    by PIL (libjpeg), then the same formula.
The expected outputs are not stored: the tests compare the GPU with oracle/sift_oracle.c on these
inputs (parity with OpenCV itself is unpinned, see sift_oracle.h).
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/data"
VIEWS = [("035_power_drill", "view_0_000"), ("035_power_drill", "view_30_004"), ("004_sugar_box", "view_60_005")]
SCENES = [("035_power_drill", "35_0010_000001"), ("006_mustard_bottle", None)]


def to_gray(rgb: np.ndarray) -> np.ndarray:
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    return ((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14).astype(np.uint8)


def main():
    out = {}
    for obj, v in VIEWS:
        col = np.asarray(Image.open(os.path.join(REF, obj, "models", v + "_color.png")).convert("RGB"))
        msk = np.asarray(Image.open(os.path.join(REF, obj, "models", v + "_mask.png")).convert("L"))
        out[f"view/{obj}/{v}"] = to_gray(col)
        out[f"mask/{obj}/{v}"] = msk
    for obj, s in SCENES:
        if s is None:
            s = sorted(os.listdir(os.path.join(REF, obj, "test_images")))[0].replace("-color.jpg", "")
        col = np.asarray(Image.open(os.path.join(REF, obj, "test_images", s + "-color.jpg")).convert("RGB"))
        out[f"scene/{obj}/{s}"] = to_gray(col)
    path = os.path.join(HERE, "sift_images.npz")
    np.savez_compressed(path, **out)
    print(path, {k: v.shape for k, v in out.items()}, os.path.getsize(path))


if __name__ == "__main__":
    main()
