"""Python mirror of the reference's hot-path interface, running on the HIP kernels of libmim.so.

Reference call sites (/root/reference/src/TestsDetector.cpp):
  :36,60   BFMatcher(NORM_L2).knnMatch(view_desc, scene_desc, knn, 2)  -> Matcher.knn_match
  :66-72   ratio test `m[0].distance < 0.9f * m[1].distance`           -> Matcher.ratio_filter
  :78      findHomography(objPts, scenePts, RANSAC, 5.0, inlierMask)   -> Matcher.find_homography
  :58-95   the per-view loop with its gates (:74, :79, :81, :84)       -> Matcher.match_batch
  :102     resize(scene, scaled, Size(), s, s) (INTER_LINEAR)          -> Matcher.resize_linear
  :106     sift->detectAndCompute(scaled, noArray(), kps, desc)        -> Matcher.sift_detect_compute
  (ModelsDetector.cpp:75, the model views with their masks: the same call with a mask)
Argument meaning and error behaviour follow OpenCV: an empty query gives no rows, n < 4 points
raise (CV_Error StsVecLengthErr), a failed RANSAC returns an empty H (None) and a zero mask.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import MimError, Params, Problem, RESULT_DTYPE

DIM = 128
# cv::KeyPoint without class_id (mim_keypoint in include/mim.h)
KEYPOINT_DTYPE = np.dtype([("x", np.float32), ("y", np.float32), ("size", np.float32), ("angle", np.float32),
                           ("response", np.float32), ("octave", np.int32)])


def default_params(**kw) -> Params:
    p = Params()
    _lib.load().mim_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


@dataclass
class DMatch:  # cv::DMatch
    queryIdx: int
    trainIdx: int
    imgIdx: int
    distance: float


class Matcher:
    """One GPU context (device + HIP stream).  Not a CPU object: construction fails without a GPU."""

    def __init__(self, device: int = 0):
        self.L = _lib.load()
        self._ctx = C.c_void_p()
        st = self.L.mim_ctx_create(device, C.byref(self._ctx))
        if st != _lib.MIM_OK:
            raise MimError(st, f"mim_ctx_create(device={device}) failed (no HIP device?)")
        self.device = device
        self._borrowed = []  # (set id, tensors) the registered sets read until they are dropped (mim.h)
        self._n_sets = 0
        self.sets_generation = 0  # bumped whenever registered sets are dropped
        self._retired = []   # (event on the matcher stream, tensors) kept alive until the event completes

    def close(self):
        if self._ctx and (self._borrowed or self._retired):
            self.L.mim_synchronize(self._ctx)
        self._borrowed, self._retired = [], []
        if self._ctx:
            self.L.mim_ctx_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int):
        if st != _lib.MIM_OK:
            raise MimError(st, self.L.mim_last_error(self._ctx).decode())

    @property
    def ctx(self):
        return self._ctx

    def set_stream(self, stream_handle: int | None):
        self._check(self.L.mim_ctx_set_stream(self._ctx, C.c_void_p(stream_handle or 0)))

    def stream_handle(self) -> int:
        """The HIP stream this matcher enqueues on (wrap with torch.cuda.ExternalStream)."""
        return int(self.L.mim_ctx_get_stream(self._ctx) or 0)

    def synchronize(self):
        self._check(self.L.mim_synchronize(self._ctx))

    # ---- descriptor sets ------------------------------------------------------------------
    def add_set(self, desc, kp) -> int:
        """Register one ObjectModel view / scene scale.  numpy (host) or torch (device) arrays.

        Device tensors are borrowed, not copied (mim.h): they must be float32, contiguous, shaped
        (n, 128) and (n, 2), on this matcher's device; the matcher keeps them alive until
        clear_sets() and orders its stream after the stream that is current when they are added."""
        on_dev = int(hasattr(desc, "is_cuda") and desc.is_cuda)
        if not on_dev:
            desc = np.ascontiguousarray(desc, np.float32).reshape(-1, DIM)
            kp = np.ascontiguousarray(kp, np.float32).reshape(-1, 2)
        else:
            import torch
            if not (hasattr(kp, "is_cuda") and kp.is_cuda):
                raise ValueError("add_set: keypoints must be on the device when the descriptors are")
            for name, t, cols in (("descriptors", desc, DIM), ("keypoints", kp, 2)):
                if t.dtype != torch.float32 or not t.is_contiguous() or t.dim() != 2 or t.shape[1] != cols:
                    raise ValueError(f"add_set: {name} must be a contiguous float32 (n, {cols}) tensor, got "
                                     f"{t.dtype} {tuple(t.shape)} contiguous={t.is_contiguous()}")
                if t.device.index != self.device:
                    raise ValueError(f"add_set: {name} on {t.device}, matcher on cuda:{self.device}")
            if kp.shape[0] != desc.shape[0]:
                raise ValueError("add_set: descriptor and keypoint row counts differ")
            # the producer stream's work (the tensors' contents) before anything on the matcher's stream
            mine = torch.cuda.ExternalStream(self.stream_handle(), device=desc.device)
            cur = torch.cuda.current_stream(desc.device)
            if cur.cuda_stream != mine.cuda_stream:
                mine.wait_stream(cur)
        n = int(desc.shape[0])
        sid = C.c_int32()
        self._check(self.L.mim_set_create(self._ctx, C.c_void_p(_lib.ptr(desc)), C.c_void_p(_lib.ptr(kp)), n,
                                          int(desc.shape[1]), on_dev, C.byref(sid)))
        if on_dev:
            self._borrowed.append((sid.value, [desc, kp]))
        self._n_sets = sid.value + 1
        return sid.value

    def add_sets(self, pairs) -> list[int]:
        """Register several sets in one library call (mim_sets_create), as add_set in order: every pair
        (desc, kp) numpy (host) or every pair torch (device), the same rules per pair; all or nothing."""
        pairs = list(pairs)
        if not pairs:
            return []
        on_dev = int(hasattr(pairs[0][0], "is_cuda") and pairs[0][0].is_cuda)
        descs, kps = [], []
        if on_dev:
            import torch
            for desc, kp in pairs:
                for name, t, cols in (("descriptors", desc, DIM), ("keypoints", kp, 2)):
                    if not (hasattr(t, "is_cuda") and t.is_cuda):
                        raise ValueError("add_sets: every array must be on the device when the first is")
                    if t.dtype != torch.float32 or not t.is_contiguous() or t.dim() != 2 or t.shape[1] != cols:
                        raise ValueError(f"add_sets: {name} must be a contiguous float32 (n, {cols}) tensor, got "
                                         f"{t.dtype} {tuple(t.shape)} contiguous={t.is_contiguous()}")
                    if t.device.index != self.device:
                        raise ValueError(f"add_sets: {name} on {t.device}, matcher on cuda:{self.device}")
                if kp.shape[0] != desc.shape[0]:
                    raise ValueError("add_sets: descriptor and keypoint row counts differ")
                descs.append(desc)
                kps.append(kp)
            dev = descs[0].device
            mine = torch.cuda.ExternalStream(self.stream_handle(), device=dev)
            cur = torch.cuda.current_stream(dev)
            if cur.cuda_stream != mine.cuda_stream:
                mine.wait_stream(cur)
        else:
            for desc, kp in pairs:
                if hasattr(desc, "is_cuda") and desc.is_cuda:
                    raise ValueError("add_sets: host and device arrays mixed")
                descs.append(np.ascontiguousarray(desc, np.float32).reshape(-1, DIM))
                kps.append(np.ascontiguousarray(kp, np.float32).reshape(-1, 2))
                if kps[-1].shape[0] != descs[-1].shape[0]:
                    raise ValueError("add_sets: descriptor and keypoint row counts differ")
        n = len(pairs)
        dp = (C.c_void_p * n)(*[_lib.ptr(d) for d in descs])
        kpp = (C.c_void_p * n)(*[_lib.ptr(k) for k in kps])
        rows = np.array([int(d.shape[0]) for d in descs], np.int32)
        first = C.c_int32()
        self._check(self.L.mim_sets_create(self._ctx, n, dp, kpp, C.c_void_p(_lib.ptr(rows)), DIM, on_dev, C.byref(first)))
        ids = list(range(first.value, first.value + n))
        if on_dev:
            for sid, d, k in zip(ids, descs, kps):
                self._borrowed.append((sid, [d, k]))
        self._n_sets = first.value + n
        return ids

    @property
    def n_sets(self) -> int:
        return self._n_sets

    def _retire(self, keep: int):
        # the dropped sets' tensors stay referenced until the work already enqueued on the matcher's
        # stream (their last readers) has completed: an event per drop, polled at the next drops
        # (not record_stream: the allocator would later record events on this stream after close())
        self._retired = [(ev, ts) for ev, ts in self._retired if not ev.query()]
        gone = [ts for sid, ts in self._borrowed if sid >= keep]
        if gone:
            import torch
            ev = torch.cuda.Event()
            ev.record(torch.cuda.ExternalStream(self.stream_handle(), device=gone[0][0].device))
            self._retired.append((ev, gone))
        self._borrowed = [(sid, ts) for sid, ts in self._borrowed if sid < keep]
        self._n_sets = min(self._n_sets, keep)
        self.sets_generation += 1

    def clear_sets(self):
        self._check(self.L.mim_sets_clear(self._ctx))
        self._retire(0)

    def truncate_sets(self, n_keep: int):
        """Drop the sets registered after the first n_keep (mim_sets_truncate); ids < n_keep stay."""
        self._check(self.L.mim_sets_truncate(self._ctx, int(n_keep)))
        self._retire(int(n_keep))

    # ---- primitives -----------------------------------------------------------------------
    def knn_match_arrays(self, query, train):
        """knnMatch(query, train, k=2) as arrays: idx (nq,2) int32 (-1 absent), dist (nq,2) float32."""
        q = np.ascontiguousarray(query, np.float32).reshape(-1, DIM)
        t = np.ascontiguousarray(train, np.float32).reshape(-1, DIM)
        nq = q.shape[0]
        idx = np.full((max(nq, 1), 2), -1, np.int32)
        dist = np.zeros((max(nq, 1), 2), np.float32)
        self._check(self.L.mim_knn2_l2(self._ctx, C.c_void_p(q.ctypes.data), nq, C.c_void_p(t.ctypes.data),
                                       t.shape[0], DIM, C.c_void_p(idx.ctypes.data), C.c_void_p(dist.ctypes.data)))
        return idx[:nq], dist[:nq]

    def knn_match(self, query, train, k: int = 2):
        """BFMatcher(NORM_L2).knnMatch(query, train, matches, k=2) -> list of lists of DMatch."""
        if k != 2:
            raise ValueError("only k=2 is on the hot path (TestsDetector.cpp:60)")
        idx, dist = self.knn_match_arrays(query, train)
        return [[DMatch(i, int(idx[i, j]), 0, float(dist[i, j])) for j in range(2) if idx[i, j] >= 0]
                for i in range(idx.shape[0])]

    # ---- feature extraction either side of the matcher (ModelsDetector.cpp:75, TestsDetector.cpp:102,106)
    def sift_detect_compute(self, gray, mask=None, max_kp: int = 1 << 18):
        """SIFT::create()->detectAndCompute(gray, mask, kps, desc) on the GPU.

        gray / mask: CV_8UC1 arrays (rows, cols).  Returns (keypoints as a KEYPOINT_DTYPE array,
        descriptors (n, 128) float32).  More than max_kp keypoints raises (no silent truncation)."""
        g = np.ascontiguousarray(gray, np.uint8)
        if g.ndim != 2:
            raise ValueError("sift_detect_compute: a single-channel image is required")
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, np.uint8)
            if m.shape != g.shape:
                raise ValueError("sift_detect_compute: mask must have the image's size")
        kps = np.zeros(max(max_kp, 1), KEYPOINT_DTYPE)
        desc = np.zeros((max(max_kp, 1), DIM), np.float32)
        n = C.c_int32()
        self._check(self.L.mim_sift_detect_compute(
            self._ctx, C.c_void_p(g.ctypes.data), g.shape[0], g.shape[1], g.strides[0],
            None if m is None else C.c_void_p(m.ctypes.data), 0 if m is None else m.strides[0], max_kp,
            C.c_void_p(kps.ctypes.data), C.c_void_p(desc.ctypes.data), C.byref(n)))
        if n.value > max_kp:
            raise ValueError(f"sift_detect_compute: {n.value} keypoints > max_kp={max_kp}")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def sift_detect_compute_scales(self, gray, scales, max_kp: int = 1 << 20):
        """resize(gray, Size(), s, s, INTER_LINEAR) + detectAndCompute at every scale in one call
        (TestsDetector.cpp:99-107).  Returns [(keypoints, descriptors)] per scale, identical to
        resize_linear + sift_detect_compute scale by scale."""
        g = np.ascontiguousarray(gray, np.uint8)
        if g.ndim != 2:
            raise ValueError("sift_detect_compute_scales: a single-channel image is required")
        sc = np.ascontiguousarray(scales, np.float32).reshape(-1)
        kps = np.zeros(max(max_kp, 1), KEYPOINT_DTYPE)
        desc = np.zeros((max(max_kp, 1), DIM), np.float32)
        n = np.zeros(len(sc), np.int32)
        self._check(self.L.mim_sift_detect_compute_scales(
            self._ctx, C.c_void_p(g.ctypes.data), g.shape[0], g.shape[1], g.strides[0], len(sc),
            C.c_void_p(sc.ctypes.data), max_kp, C.c_void_p(kps.ctypes.data), C.c_void_p(desc.ctypes.data),
            C.c_void_p(n.ctypes.data)))
        out, o = [], 0
        for c in n:
            out.append((kps[o:o + c].copy(), desc[o:o + c].copy()))
            o += int(c)
        return out

    def sift_scales_to_sets(self, gray, scales, keypoints: bool = False, max_kp: int = 1 << 20):
        """resize + detectAndCompute at every scale (TestsDetector.cpp:99-107) with the descriptors left
        on the device, each scale registered as a set (mim_sift_scales_sets).  Returns (set ids, n_kp
        per scale, [keypoints per scale] or None); the sets' rows are what sift_detect_compute_scales
        returns, without the round trip through host memory.  With keypoints=True and more than max_kp
        keypoints in all, this call's sets are dropped and the call made again with room for all."""
        g = np.ascontiguousarray(gray, np.uint8)
        if g.ndim != 2:
            raise ValueError("sift_scales_to_sets: a single-channel image is required")
        sc = np.ascontiguousarray(scales, np.float32).reshape(-1)
        ids = np.zeros(len(sc), np.int32)
        n = np.zeros(len(sc), np.int32)
        kps = np.zeros(max(max_kp, 1), KEYPOINT_DTYPE) if keypoints else None
        before = self.sets_info()[0]
        st = self.L.mim_sift_scales_sets(
            self._ctx, C.c_void_p(g.ctypes.data), g.shape[0], g.shape[1], g.strides[0], len(sc),
            C.c_void_p(sc.ctypes.data), C.c_void_p(ids.ctypes.data), C.c_void_p(n.ctypes.data),
            max_kp if keypoints else 0, C.c_void_p(kps.ctypes.data) if keypoints else None)
        # the context's set count, whatever happened (MIM_ERANGE for a short host keypoint buffer comes
        # after the sets were registered)
        self._n_sets = self.sets_info()[0]
        if st == _lib.MIM_ERANGE and keypoints and self._n_sets == before + len(sc) and int(n.sum()) > max_kp:
            self.truncate_sets(before)  # drop this call's sets, run again with room for all
            return self.sift_scales_to_sets(gray, scales, True, int(n.sum()))
        self._check(st)
        out = None
        if keypoints:
            out, o = [], 0
            for c in n:
                out.append(kps[o:o + c].copy())
                o += int(c)
        return [int(i) for i in ids], [int(c) for c in n], out

    def sets_info(self):
        """(registered set count, sets generation) of the context (mim_sets_info)."""
        n, gen = C.c_int32(), C.c_int64()
        self._check(self.L.mim_sets_info(self._ctx, C.byref(n), C.byref(gen)))
        return n.value, gen.value

    def set_rows(self, set_id: int):
        """The descriptor rows (n, 128) float32 and keypoint positions (n, 2) of a registered set as the
        kernels read them (mim_set_rows; a debug/test copy-out, e.g. of mim_sift_scales_sets' sets)."""
        n = C.c_int32()
        self._check(self.L.mim_set_rows(self._ctx, int(set_id), 0, None, None, C.byref(n)))
        desc = np.zeros((n.value, DIM), np.float32)
        kp = np.zeros((n.value, 2), np.float32)
        if n.value:
            self._check(self.L.mim_set_rows(self._ctx, int(set_id), n.value, C.c_void_p(desc.ctypes.data),
                                            C.c_void_p(kp.ctypes.data), C.byref(n)))
        return desc, kp

    def resize_linear(self, src, dsize=None, fx: float = 0.0, fy: float = 0.0):
        """cv::resize(src, dst, dsize, fx, fy, INTER_LINEAR) of a CV_8UC1 image.

        dsize = (width, height), or None with fx (and fy, default fx) > 0 as the reference calls it:
        resize(scene, scaled, Size(), scale, scale) with a float scale (TestsDetector.cpp:99-102)."""
        s = np.ascontiguousarray(src, np.uint8)
        if dsize is None:
            if not fx > 0:
                raise ValueError("resize_linear: dsize or fx > 0 required")
            fx = float(np.float32(fx))
            fy = float(np.float32(fy)) if fy else fx
            dcols, drows = int(np.rint(s.shape[1] * fx)), int(np.rint(s.shape[0] * fy))
        else:
            dcols, drows = int(dsize[0]), int(dsize[1])
            fx = fy = 0.0
        dst = np.zeros((max(drows, 1), max(dcols, 1)), np.uint8)
        self._check(self.L.mim_resize_linear_u8(self._ctx, C.c_void_p(s.ctypes.data), s.shape[0], s.shape[1],
                                                s.strides[0], C.c_void_p(dst.ctypes.data), drows, dcols, fx, fy))
        return dst

    def ratio_filter(self, idx, dist, ratio: float = 0.9):
        idx = np.ascontiguousarray(idx, np.int32)
        dist = np.ascontiguousarray(dist, np.float32)
        nq = idx.shape[0]
        qo = np.zeros(max(nq, 1), np.int32)
        to = np.zeros(max(nq, 1), np.int32)
        ng = C.c_int32()
        self._check(self.L.mim_ratio_filter(self._ctx, C.c_void_p(idx.ctypes.data), C.c_void_p(dist.ctypes.data),
                                            nq, ratio, C.c_void_p(qo.ctypes.data), C.c_void_p(to.ctypes.data),
                                            C.byref(ng)))
        return qo[:ng.value], to[:ng.value]

    def find_homography(self, src, dst, thresh: float = 5.0, max_iters: int = 2000, confidence: float = 0.995):
        """cv::findHomography(src, dst, RANSAC, thresh, mask, max_iters, confidence) -> (H or None, mask)."""
        src = np.ascontiguousarray(src, np.float32).reshape(-1, 2)
        dst = np.ascontiguousarray(dst, np.float32).reshape(-1, 2)
        n = src.shape[0]
        if n < 4 or dst.shape[0] != n:
            raise ValueError("The input arrays should have at least 4 corresponding point sets to calculate Homography")
        H = np.zeros(9, np.float64)
        mask = np.zeros(n, np.uint8)
        st = self.L.mim_find_homography(self._ctx, C.c_void_p(src.ctypes.data), C.c_void_p(dst.ctypes.data), n,
                                        thresh, max_iters, confidence, C.c_void_p(H.ctypes.data),
                                        C.c_void_p(mask.ctypes.data))
        if st == _lib.MIM_ENOMODEL:
            return None, mask
        self._check(st)
        return H.reshape(3, 3), mask

    # ---- fused batch ----------------------------------------------------------------------
    def match_batch_async(self, problems, params: Params | None = None):
        params = params or default_params()
        # an (n, 2) int32 array is mim_problem[n] as it is (no per-problem ctypes objects: ~1 us each)
        arr = problems if isinstance(problems, np.ndarray) else np.asarray(list(problems), np.int32)
        arr = np.ascontiguousarray(arr, np.int32).reshape(-1, 2)
        self._check(self.L.mim_batch_run(self._ctx, arr.ctypes.data_as(C.POINTER(Problem)), len(arr),
                                         C.byref(params)))
        return len(arr)

    def batch_results(self, n: int) -> np.ndarray:
        """Waits for the last batch and returns its n records (n must be the batch's problem count;
        n = 0 only waits and collects the kernel timings)."""
        out = np.zeros(n, RESULT_DTYPE)
        self._check(self.L.mim_batch_results(self._ctx, C.c_void_p(out.ctypes.data if n else 0)))
        return out

    def batch_results_copy_to(self, dst_dev):
        """Async device-to-device copy of the last batch's records (for an RCCL gather)."""
        self._check(self.L.mim_batch_results_copy(self._ctx, C.c_void_p(_lib.ptr(dst_dev)), 1))

    def batch_results_dev_ptr(self) -> int:
        return int(self.L.mim_batch_results_dev(self._ctx) or 0)

    def problem_detail(self, i: int, n_good: int):
        q = np.zeros(max(n_good, 1), np.int32)
        t = np.zeros(max(n_good, 1), np.int32)
        m = np.zeros(max(n_good, 1), np.uint8)
        self._check(self.L.mim_batch_problem_detail(self._ctx, i, C.c_void_p(q.ctypes.data), C.c_void_p(t.ctypes.data),
                                                    C.c_void_p(m.ctypes.data)))
        return q[:n_good], t[:n_good], m[:n_good]

    def batch_inlier_points(self, n: int, scales=None):
        """allUnfilteredScenePts of the last batch (mim_batch_inlier_points, TestsDetector.cpp:87-94):
        (offsets (n + 1,) int64, points (offsets[n], 2) float32); problem i's inlier scene points, divided
        by scales[i] when it is not 1, are points[offsets[i]:offsets[i + 1]]."""
        offs = np.zeros(n + 1, np.int64)
        sc = None if scales is None else np.ascontiguousarray(scales, np.float32)
        if sc is not None and sc.shape != (n,):
            raise ValueError(f"batch_inlier_points: {sc.shape} scales for {n} problems")
        scp = None if sc is None else sc.ctypes.data_as(C.POINTER(C.c_float))
        op = offs.ctypes.data_as(C.POINTER(C.c_int64))
        # one call into a kept buffer (one wait, one gather); a larger total comes back as MIM_ERANGE with
        # the offsets set, and the call is made again with room for all
        buf = getattr(self, "_inl_buf", None)
        if buf is None:
            buf = self._inl_buf = np.zeros((1 << 16, 2), np.float32)
        st = self.L.mim_batch_inlier_points(self._ctx, scp, buf.ctypes.data_as(C.POINTER(C.c_float)), buf.shape[0], op)
        total = int(offs[n])
        if st == _lib.MIM_ERANGE and total > buf.shape[0]:
            buf = self._inl_buf = np.zeros((2 * total, 2), np.float32)
            st = self.L.mim_batch_inlier_points(self._ctx, scp, buf.ctypes.data_as(C.POINTER(C.c_float)), buf.shape[0], op)
        self._check(st)
        return offs, buf[:total].copy()

    def match_batch(self, problems, params: Params | None = None) -> np.ndarray:
        n = self.match_batch_async(problems, params)
        return self.batch_results(n)

    def knn_sets_dev(self, qset: int, tset: int, idx_dev, dist_dev):
        self._check(self.L.mim_knn2_sets_dev(self._ctx, qset, tset, C.c_void_p(_lib.ptr(idx_dev)),
                                             C.c_void_p(_lib.ptr(dist_dev))))

    def set_sampler_stream(self, on: bool):
        """Second-stream getSubset replay (mim_ctx_set_sampler_stream): on for a batch alone, off when
        several contexts already overlap their batches."""
        self._check(self.L.mim_ctx_set_sampler_stream(self._ctx, int(on)))

    def set_timing(self, on: bool):
        self._check(self.L.mim_set_timing(self._ctx, int(on)))

    def kernel_ms(self, name: str) -> float:
        return float(self.L.mim_last_kernel_ms(self._ctx, name.encode()))
