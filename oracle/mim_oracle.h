/*
 * mim_oracle.h — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline.  The product (libmim.so) never links it.
 *
 * What it restates (reference call sites, /root/reference):
 *   src/TestsDetector.cpp:36,60   BFMatcher(NORM_L2).knnMatch(q, t, m, 2)      -> orc_knn2_l2
 *   src/TestsDetector.cpp:66-72   ratio test d0 < 0.9f*d1, ordered gather      -> orc_ratio_filter
 *   src/TestsDetector.cpp:78      findHomography(obj, scene, RANSAC, 5.0, mask) -> orc_find_homography
 *   src/TestsDetector.cpp:74-94   gates, det filter, inlier gather              -> orc_match_problem
 * The arithmetic lives in OpenCV (not vendored, not installed here, version unpinned; restatement
 * target OpenCV 4.5.4 = Ubuntu 22.04 libopencv-dev).
 *
 * PARITY STATUS: "parity partially pinned".  The reference ships no tests, fixtures or golden
 * vectors for this path and OpenCV cannot be built or imported in this image, so the restatement
 * is pinned only by analytic known-answer tests (tests/test_oracle_kat.py: MWC RNG sequence,
 * RANSACUpdateNumIters table, exact homography recovery, planted nearest neighbours, ratio/tie
 * boundaries) and by the reference's own constants (TestsDetector.cpp:21-25).
 * cv::eigen is restated on OpenCV's JacobiImpl_ path (the non-HAVE_EIGEN build), see DESIGN.md.
 */
#ifndef MIM_ORACLE_H
#define MIM_ORACLE_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

/* cv::RNG (core/include/opencv2/core/operations.hpp): multiply-with-carry, coefficient 4164903690 */
uint32_t orc_rng_next(uint64_t* state);
/* Fill out[0..n) with the raw next() stream of RNG((uint64)-1) — what every findHomography call sees. */
void orc_rng_stream(uint64_t seed, uint32_t* out, int64_t n);

/* batchDistance(NORM_L2, K=2) semantics: idx[2*i+k] / dist[2*i+k], -1 / FLT_MAX when absent.
 * d = sqrtf(normL2Sqr_) with OpenCV's SSE accumulation order (4 accumulators x 4 lanes).
 * nthreads <= 0 -> all cores (OpenCV parallel_for_ over query rows). */
void orc_knn2_l2(const float* q, int nq, const float* t, int nt, int dim,
                 int32_t* idx, float* dist, int nthreads);

/* TestsDetector.cpp:66-72: keep query i iff it has 2 matches and d0 < ratio*d1; writes query and
 * train indices of the kept matches in ascending query order, returns the count. */
int orc_ratio_filter(const int32_t* idx, const float* dist, int nq, float ratio,
                     int32_t* q_out, int32_t* t_out);

/* calib3d pieces, exposed for known-answer tests */
int orc_update_num_iters(double p, double ep, int model_points, int max_iters);
int orc_have_collinear(const float* xy, int count);
int orc_check_subset(const float* src4, const float* dst4);
int orc_run_kernel(const float* src, const float* dst, int n, double H[9]);
void orc_jacobi(double* A, double* W, double* V, int n); /* A, V row-major n*n; eigvecs in V rows */
void orc_compute_error(const float* src, const float* dst, int n, const double H[9], float* err);

/* RANSACPointSetRegistrator::run with the HomographyEstimatorCallback.
 * Returns 1 on success.  H = best minimal-sample model, mask = best mask, *n_iters = iterations
 * executed, *best_iter = iteration that produced the best model, *stream_used = RNG draws. */
int orc_ransac(const float* src, const float* dst, int n, double thresh, double conf, int max_iters,
               double H[9], uint8_t* mask, int* n_iters, int* best_iter, int64_t* stream_used);

/* cv::findHomography(src, dst, RANSAC, thresh, mask, max_iters, conf): RANSAC + refit on the
 * inliers + Levenberg-Marquardt refine (10 iters).  Returns 1 if H is non-empty. */
int orc_find_homography(const float* src, const float* dst, int n, double thresh, int max_iters,
                        double conf, double H[9], uint8_t* mask);

/* One (model view, scene scale) problem, TestsDetector.cpp:58-95. */
typedef struct {
    float ratio;            /* 0.9f  TestsDetector.cpp:21 */
    int32_t min_good;       /* 4     :22 / :74 */
    int32_t min_inliers;    /* 4     :22 / :81 */
    double ransac_thresh;   /* 5.0   :23 */
    int32_t max_iters;      /* 2000  findHomography default */
    double confidence;      /* 0.995 findHomography default */
    double det_lo, det_hi;  /* (double)0.1f, (double)10.0f  :24-25,:84 */
} orc_params;

typedef struct {
    int32_t n_good;     /* matches surviving the ratio test */
    int32_t n_inl;      /* countNonZero(mask) */
    int32_t status;     /* 0 accepted, 1 few good, 2 empty H, 3 few inliers, 4 det out of range */
    int32_t iters;      /* RANSAC iterations executed */
    double H[9];
    double det;
} orc_result;

/* Study knob, off by default (tools/eigen_gap.py): perturb every minimal-sample model of orc_ransac by
 * up to +-ulps ulp per element, modelling an OpenCV whose cv::eigen is Eigen's solver. */
void orc_set_model_perturbation(int ulps, uint64_t seed);
/* Study knob: orc_ransac writes each iteration's inlier count (-1 = degenerate sample) to counts[iter]
 * for iter < cap; NULL turns it off.  Not thread-safe (one process per study worker). */
void orc_set_count_trace(int* counts, int cap);

void orc_default_params(orc_params* p);
/* Full per-problem path.  mask_out (optional) receives n_good bytes. good_q/good_t optional
 * (n_q ints each) receive the ratio-test survivors. knn_threads as in orc_knn2_l2. */
void orc_match_problem(const float* qdesc, const float* qkp, int nq,
                       const float* tdesc, const float* tkp, int nt, int dim,
                       const orc_params* prm, int knn_threads, orc_result* res,
                       uint8_t* mask_out, int32_t* good_q, int32_t* good_t);

#ifdef __cplusplus
}
#endif
#endif
