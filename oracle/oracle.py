"""ctypes view of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker or the timed CPU baseline.  See oracle/mim_oracle.h for what the C code
restates (reference call sites TestsDetector.cpp:60,66-72,78) and its parity-pinning status
("parity partially pinned": KATs only — OpenCV is absent and the reference ships no fixtures).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_lib = None


class Params(C.Structure):
    _fields_ = [("ratio", C.c_float), ("min_good", C.c_int32), ("min_inliers", C.c_int32),
                ("ransac_thresh", C.c_double), ("max_iters", C.c_int32), ("confidence", C.c_double),
                ("det_lo", C.c_double), ("det_hi", C.c_double)]


class Result(C.Structure):
    _fields_ = [("n_good", C.c_int32), ("n_inl", C.c_int32), ("status", C.c_int32),
                ("iters", C.c_int32), ("H", C.c_double * 9), ("det", C.c_double)]


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", _HERE])
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        f32p, i32p, u8p, f64p = (np.ctypeslib.ndpointer(np.float32, flags="C"),
                                 np.ctypeslib.ndpointer(np.int32, flags="C"),
                                 np.ctypeslib.ndpointer(np.uint8, flags="C"),
                                 np.ctypeslib.ndpointer(np.float64, flags="C"))
        L.orc_rng_stream.argtypes = [C.c_uint64, np.ctypeslib.ndpointer(np.uint32, flags="C"), C.c_int64]
        L.orc_knn2_l2.argtypes = [f32p, C.c_int, f32p, C.c_int, C.c_int, i32p, f32p, C.c_int]
        L.orc_ratio_filter.argtypes = [i32p, f32p, C.c_int, C.c_float, i32p, i32p]
        L.orc_ratio_filter.restype = C.c_int
        L.orc_update_num_iters.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int]
        L.orc_update_num_iters.restype = C.c_int
        L.orc_have_collinear.argtypes = [f32p, C.c_int]
        L.orc_check_subset.argtypes = [f32p, f32p]
        L.orc_run_kernel.argtypes = [f32p, f32p, C.c_int, f64p]
        L.orc_jacobi.argtypes = [f64p, f64p, f64p, C.c_int]
        L.orc_compute_error.argtypes = [f32p, f32p, C.c_int, f64p, f32p]
        L.orc_ransac.argtypes = [f32p, f32p, C.c_int, C.c_double, C.c_double, C.c_int, f64p, u8p,
                                 C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int64)]
        L.orc_find_homography.argtypes = [f32p, f32p, C.c_int, C.c_double, C.c_int, C.c_double, f64p, u8p]
        L.orc_default_params.argtypes = [C.POINTER(Params)]
        L.orc_set_model_perturbation.argtypes = [C.c_int, C.c_uint64]
        L.orc_set_count_trace.argtypes = [C.c_void_p, C.c_int]
        L.orc_match_problem.argtypes = [f32p, f32p, C.c_int, f32p, f32p, C.c_int, C.c_int,
                                        C.POINTER(Params), C.c_int, C.POINTER(Result),
                                        C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_resize_linear_u8.argtypes = [u8p, C.c_int, C.c_int, u8p, C.c_int, C.c_int, C.c_double, C.c_double]
        L.orc_sift_detect_compute.argtypes = [u8p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.orc_sift_detect_compute.restype = C.c_int
        L.orc_fast_atan2.argtypes = [C.c_float, C.c_float]
        L.orc_fast_atan2.restype = C.c_float
        _lib = L
    return _lib


def rng_stream(n: int, seed: int = 0xFFFFFFFFFFFFFFFF) -> np.ndarray:
    out = np.empty(n, np.uint32)
    lib().orc_rng_stream(seed, out, n)
    return out


def knn2(q: np.ndarray, t: np.ndarray, threads: int = 0):
    q = np.ascontiguousarray(q, np.float32)
    t = np.ascontiguousarray(t, np.float32)
    nq = q.shape[0]
    idx = np.full((max(nq, 1), 2), -1, np.int32)
    dist = np.zeros((max(nq, 1), 2), np.float32)
    lib().orc_knn2_l2(q, nq, t, t.shape[0], q.shape[1] if q.ndim == 2 else 128, idx, dist, threads)
    return idx[:nq], dist[:nq]


def ratio_filter(idx, dist, ratio=0.9):
    nq = idx.shape[0]
    qo = np.zeros(max(nq, 1), np.int32)
    to = np.zeros(max(nq, 1), np.int32)
    n = lib().orc_ratio_filter(np.ascontiguousarray(idx, np.int32), np.ascontiguousarray(dist, np.float32),
                               nq, ratio, qo, to)
    return qo[:n], to[:n]


def update_num_iters(p, ep, model_points, max_iters):
    return lib().orc_update_num_iters(p, ep, model_points, max_iters)


def run_kernel(src, dst):
    H = np.zeros(9, np.float64)
    r = lib().orc_run_kernel(np.ascontiguousarray(src, np.float32), np.ascontiguousarray(dst, np.float32),
                             len(src), H)
    return r, H.reshape(3, 3)


def check_subset(src4, dst4):
    return lib().orc_check_subset(np.ascontiguousarray(src4, np.float32), np.ascontiguousarray(dst4, np.float32))


def jacobi(A):
    A = np.array(A, np.float64, copy=True, order="C")
    n = A.shape[0]
    W = np.zeros(n)
    V = np.zeros((n, n))
    lib().orc_jacobi(A, W, V, n)
    return W, V


def compute_error(src, dst, H):
    err = np.zeros(len(src), np.float32)
    lib().orc_compute_error(np.ascontiguousarray(src, np.float32), np.ascontiguousarray(dst, np.float32),
                            len(src), np.ascontiguousarray(H, np.float64).reshape(9), err)
    return err


def ransac(src, dst, thresh=5.0, conf=0.995, max_iters=2000):
    n = len(src)
    H = np.zeros(9)
    mask = np.zeros(max(n, 1), np.uint8)
    it, bi, used = C.c_int(0), C.c_int(0), C.c_int64(0)
    ok = lib().orc_ransac(np.ascontiguousarray(src, np.float32), np.ascontiguousarray(dst, np.float32),
                          n, thresh, conf, max_iters, H, mask, C.byref(it), C.byref(bi), C.byref(used))
    return dict(ok=ok, H=H.reshape(3, 3), mask=mask[:n], iters=it.value, best_iter=bi.value,
                stream_used=used.value)


def set_model_perturbation(ulps: int, seed: int = 0):
    """Study knob (tools/eigen_gap.py): +-ulps ulp on every minimal-sample model; 0 = off."""
    lib().orc_set_model_perturbation(int(ulps), int(seed) & 0xFFFFFFFFFFFFFFFF)


def ransac_counts(src, dst, thresh=5.0, conf=0.995, max_iters=2000):
    """orc_ransac with the per-iteration inlier counts (study knob): (result dict, counts[:iters])."""
    counts = np.full(max(max_iters, 1), -2, np.int32)
    lib().orc_set_count_trace(counts.ctypes.data, len(counts))
    try:
        r = ransac(src, dst, thresh, conf, max_iters)
    finally:
        lib().orc_set_count_trace(None, 0)
    return r, counts[:r["iters"]]


def find_homography(src, dst, thresh=5.0, max_iters=2000, conf=0.995):
    n = len(src)
    H = np.zeros(9)
    mask = np.zeros(max(n, 1), np.uint8)
    ok = lib().orc_find_homography(np.ascontiguousarray(src, np.float32), np.ascontiguousarray(dst, np.float32),
                                   n, thresh, max_iters, conf, H, mask)
    return ok, H.reshape(3, 3), mask[:n]


def default_params(**kw) -> Params:
    p = Params()
    lib().orc_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def match_problem(qd, qk, td, tk, params: Params | None = None, threads: int = 0):
    params = params or default_params()
    qd = np.ascontiguousarray(qd, np.float32)
    td = np.ascontiguousarray(td, np.float32)
    qk = np.ascontiguousarray(qk, np.float32)
    tk = np.ascontiguousarray(tk, np.float32)
    nq = qd.shape[0]
    res = Result()
    mask = np.zeros(max(nq, 1), np.uint8)
    gq = np.zeros(max(nq, 1), np.int32)
    gt = np.zeros(max(nq, 1), np.int32)
    lib().orc_match_problem(qd, qk, nq, td, tk, td.shape[0], 128, C.byref(params), threads, C.byref(res),
                            mask.ctypes.data, gq.ctypes.data, gt.ctypes.data)
    ng = res.n_good
    return dict(n_good=ng, n_inl=res.n_inl, status=res.status, iters=res.iters,
                H=np.array(res.H[:]).reshape(3, 3), det=res.det,
                mask=mask[:ng] if ng >= params.min_good else np.zeros(0, np.uint8),
                good_q=gq[:ng], good_t=gt[:ng])


# ---- SIFT / resize (sift_oracle.h; ModelsDetector.cpp:75, TestsDetector.cpp:102,106) ----------
KEYPOINT_DTYPE = np.dtype([("x", np.float32), ("y", np.float32), ("size", np.float32), ("angle", np.float32),
                           ("response", np.float32), ("octave", np.int32)])


def resize_dsize(rows: int, cols: int, fx: float, fy: float):
    """dsize of resize(src, dst, Size(), fx, fy): saturate_cast<int>(cols * fx) (round half even)."""
    return int(np.rint(cols * float(fx))), int(np.rint(rows * float(fy)))


def resize_linear_u8(src: np.ndarray, dsize=None, fx: float = 0.0, fy: float = 0.0) -> np.ndarray:
    """cv::resize(src, dst, dsize, fx, fy, INTER_LINEAR) of a CV_8UC1 image; dsize = (width, height) or
    None with fx, fy > 0 (float factors as the reference passes them, TestsDetector.cpp:99-102)."""
    src = np.ascontiguousarray(src, np.uint8)
    if dsize is None:
        fx = float(np.float32(fx))
        fy = float(np.float32(fy)) if fy else fx
        dsize = resize_dsize(src.shape[0], src.shape[1], fx, fy)
    else:
        fx = fy = 0.0
    dcols, drows = dsize
    dst = np.zeros((drows, dcols), np.uint8)
    lib().orc_resize_linear_u8(src, src.shape[0], src.shape[1], dst, drows, dcols, fx, fy)
    return dst


def sift_detect_compute(gray: np.ndarray, mask: np.ndarray | None = None, max_kp: int = 1 << 20):
    """SIFT::create()->detectAndCompute(gray, mask): (keypoints [KEYPOINT_DTYPE], descriptors (n,128) f32)."""
    gray = np.ascontiguousarray(gray, np.uint8)
    m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    kps = np.zeros(max_kp, KEYPOINT_DTYPE)
    desc = np.zeros((max_kp, 128), np.float32)
    n = lib().orc_sift_detect_compute(gray, gray.shape[0], gray.shape[1], None if m is None else m.ctypes.data,
                                      max_kp, kps.ctypes.data, desc.ctypes.data)
    n = min(n, max_kp)
    return kps[:n].copy(), desc[:n].copy()


def fast_atan2(y: float, x: float) -> float:
    return float(lib().orc_fast_atan2(y, x))
