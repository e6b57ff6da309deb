/* sift_oracle.h — CPU restatement of OpenCV 4.5.4 SIFT::detectAndCompute (default parameters) and of
 * resize(INTER_LINEAR) on 8-bit images — TEST INFRASTRUCTURE ONLY (checker of csrc/sift.hip).
 *
 * Reference call sites: /root/reference/src/ModelsDetector.cpp:75 (model views, with mask),
 * /root/reference/src/TestsDetector.cpp:102,106 (scene scales: resize then detectAndCompute), with
 * SIFT::create() defaults (main.cpp:17): nfeatures 0, nOctaveLayers 3, contrastThreshold 0.04,
 * edgeThreshold 10, sigma 1.6, CV_32F descriptors.
 *
 * OpenCV is not in this image, so this restates the recalled OpenCV routines (features2d
 * sift.simd.hpp / sift.dispatch.cpp, imgproc resize.cpp / smooth.dispatch.cpp / filter, core
 * fastAtan2) in scalar float arithmetic, compiled -ffp-contract=off.  Parity against OpenCV itself is
 * UNPINNED.  Transcendentals: OpenCV's cv::hal::exp32f approximation (not restated) and libm's
 * expf/powf/sinf/cosf are all replaced by the double-precision function rounded to float — what the
 * GPU computes too, so the two agree except where a result sits within ~1e-16 of a float rounding
 * boundary.  fastAtan2 is OpenCV's polynomial, sqrt and division IEEE.  Summation orders: Gaussian row
 * pass sequential over the taps, column pass in OpenCV's symmetric grouping, histograms in pixel order.
 */
#ifndef MIM_SIFT_ORACLE_H
#define MIM_SIFT_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    float x, y, size, angle, response;
    int32_t octave;
} orc_keypoint; /* cv::KeyPoint (class_id unused) */

/* cv::resize(src, dst, dsize, fx, fy, INTER_LINEAR) for CV_8UC1 (fixed-point path).  fx, fy > 0: the
 * factors of resize(src, dst, Size(), fx, fy) (TestsDetector.cpp:102), drows / dcols then being
 * cvRound(rows * fy) / cvRound(cols * fx); fx, fy = 0: dsize given, factors dcols / cols, drows / rows. */
void orc_resize_linear_u8(const uint8_t* src, int rows, int cols, uint8_t* dst, int drows, int dcols, double fx,
                          double fy);

/* SIFT::detectAndCompute(img, mask, kps, desc): img CV_8UC1 rows x cols (row stride = cols), mask
 * (nullable) CV_8UC1 of the same size.  Writes at most max_kp keypoints + 128-float descriptors and
 * returns the number found (may exceed max_kp: only the first max_kp are written). */
int orc_sift_detect_compute(const uint8_t* img, int rows, int cols, const uint8_t* mask, int max_kp,
                            orc_keypoint* kps, float* desc);

/* OpenCV's fastAtan2 (degrees, polynomial approximation), for the KAT tests. */
float orc_fast_atan2(float y, float x);

#ifdef __cplusplus
}
#endif
#endif
