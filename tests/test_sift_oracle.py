"""CPU checks of the SIFT / resize restatement (oracle/sift_oracle.c), the checker of csrc/sift.hip.

OpenCV is absent and the reference ships no SIFT outputs, so parity with OpenCV is unpinned; these
are the analytic known-answer properties the restatement must satisfy.
"""
import numpy as np
import pytest


def blob(rows, cols, cy, cx, s, amp=120.0, base=60.0):
    y, x = np.mgrid[0:rows, 0:cols].astype(np.float64)
    return np.clip(np.rint(base + amp * np.exp(-((y - cy) ** 2 + (x - cx) ** 2) / (2 * s * s))), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("y,x,deg", [(0, 1, 0), (1, 1, 45), (1, 0, 90), (0, -1, 180), (-1, 0, 270), (-1, 1, 315)])
def test_fast_atan2(oracle, y, x, deg):
    assert abs(oracle.fast_atan2(y, x) - deg) < 0.01


def test_resize_identity_and_constant(oracle):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (33, 47), dtype=np.uint8)
    assert np.array_equal(oracle.resize_linear_u8(img, (47, 33)), img)
    c = np.full((40, 50), 77, np.uint8)
    for s in (0.7, 0.85, 1.15, 1.3):
        r = oracle.resize_linear_u8(c, fx=s)
        assert np.all(r == 77), s


def test_resize_dsize_rounding(oracle):
    # Size() with fx = fy = scale: dsize = cvRound(cols * scale), cvRound(rows * scale) (TestsDetector.cpp:102)
    img = np.zeros((480, 640), np.uint8)
    for s, shape in ((0.7, (336, 448)), (0.85, (408, 544)), (1.15, (552, 736)), (1.3, (624, 832))):
        assert oracle.resize_linear_u8(img, fx=s).shape == shape


def test_resize_half_is_pair_average(oracle):
    # x 0.5: source position 2d + 0.5, weights 1/2 each: the rounded mean of each 2 x 2 block
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (32, 48), dtype=np.uint8)
    r = oracle.resize_linear_u8(img, fx=0.5).astype(np.int64)
    blocks = img.reshape(16, 2, 24, 2).astype(np.int64).sum(axis=(1, 3))
    assert np.abs(r * 4 - blocks).max() <= 3


def test_sift_flat_and_masked(oracle):
    k, d = oracle.sift_detect_compute(np.full((64, 64), 100, np.uint8))
    assert len(k) == 0 and d.shape == (0, 128)
    img = blob(96, 96, 48, 48, 6)
    k, _ = oracle.sift_detect_compute(img, np.zeros_like(img))
    assert len(k) == 0


def test_sift_blob_keypoint(oracle):
    """A single isotropic blob: a keypoint at its centre whose scale follows the blob's sigma."""
    for s in (4.0, 6.0):
        img = blob(128, 128, 64.3, 63.6, s)
        k, d = oracle.sift_detect_compute(img)
        assert len(k) >= 1
        c = np.hypot(k["x"] - 63.6, k["y"] - 64.3)
        i = int(np.argmin(c))
        assert c[i] < 0.5
        # DoG extremum of a Gaussian blob of sigma s: keypoint size (diameter) ~ 2 * sqrt(2) * s
        assert 0.5 * 2.8 * s < k["size"][i] < 2.0 * 2.8 * s
        assert d.shape == (len(k), 128) and np.array_equal(d, np.rint(d)) and d.max() <= 255 and d.min() >= 0


def test_sift_octave_packing_and_order(oracle):
    rng = np.random.default_rng(3)
    img = np.clip(rng.normal(128, 40, (120, 160)), 0, 255).astype(np.uint8)
    img = oracle.resize_linear_u8(oracle.resize_linear_u8(img, fx=0.5), (160, 120))  # smooth it
    k, _ = oracle.sift_detect_compute(img)
    assert len(k) > 5
    octv = k["octave"] & 255
    octv = np.where(octv < 128, octv, octv - 256)
    layer = (k["octave"] >> 8) & 255
    assert octv.min() >= -1 and 1 <= layer.min() and layer.max() <= 3
    order = np.lexsort((-k["octave"], -k["response"], -k["angle"], -k["size"], -k["y"], -k["x"]))
    assert np.array_equal(order, np.arange(len(k)))  # KeypointGreater (sorted, deduplicated)


def test_sift_rotation_90(oracle):
    """Rotating the image by 90 degrees maps the blob keypoint and rotates its angle by 90 degrees
    (up to the orientation histogram's interpolation); descriptors stay close."""
    img = blob(96, 96, 40, 52, 5) // 2 + blob(96, 96, 47, 52, 3, amp=80, base=0) // 2
    r = np.ascontiguousarray(np.rot90(img))  # counter-clockwise: (y, x) -> (95 - x, y)
    k0, d0 = oracle.sift_detect_compute(img)
    k1, d1 = oracle.sift_detect_compute(r)
    assert len(k0) > 0 and len(k1) > 0
    i = int(np.argmax(k0["response"]))
    px, py = k0["y"][i], 95 - k0["x"][i]
    j = int(np.argmin(np.hypot(k1["x"] - px, k1["y"] - py) + 1000 * (np.abs(k1["size"] - k0["size"][i]) > 0.5)))
    assert np.hypot(k1["x"][j] - px, k1["y"][j] - py) < 0.5
    da = (k1["angle"][j] - k0["angle"][i]) % 360
    assert min(abs(da - 90), abs(da - 270)) < 5 or min(da, 360 - da) < 5 or abs(da - 180) < 5
