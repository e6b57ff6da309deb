// mim_internal.h — device-side data layout shared by the HIP kernels and the host launcher.
// See DESIGN.md "Data layout in HBM".  gfx950 only (wave64, i8 MFMA 32x32x32, f16/fp64 RANSAC).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mim {

constexpr int kDim = 128;          // SIFT descriptor length (TestsDetector.cpp:60 operands)
constexpr int kTileRows = 64;      // descriptor rows per staged tile
constexpr int kTileBytes = kTileRows * kDim;  // 8 KiB of i8 per tile
constexpr int kNormWords = 4 * kTileRows;      // norm block per tile (knn.hip prep_tile)
constexpr int kWave = 64;
#ifndef MIM_KNN_QT
#define MIM_KNN_QT 2
#endif

#ifndef MIM_KNN_WAVES
#define MIM_KNN_WAVES 8
#endif
#ifndef MIM_KNN_STAGE
#define MIM_KNN_STAGE 4
#endif
constexpr int kKnnQT = MIM_KNN_QT;             // 32-query MFMA column tiles per wave (distance kernel)
constexpr int kKnnWaves = MIM_KNN_WAVES;       // waves per distance-kernel block
constexpr int kKnnStage = MIM_KNN_STAGE;       // 64-row train tiles per LDS stage (per barrier)
constexpr int kKnnMinChunk = 8;                // fewest train tiles per distance-kernel block
#ifndef MIM_KNN_SUB_TILES
#define MIM_KNN_SUB_TILES -1
#endif
constexpr int kKnnSubTiles = MIM_KNN_SUB_TILES;  // distance schedule's sub-chunk target (api.cpp build_tables)
constexpr int kKnnBlockQ = kKnnWaves * 32 * kKnnQT;  // queries per distance-kernel work item

// One descriptor set = one ObjectModel view (objectModel.hpp:11-16) or one scaled scene
// (TestsDetector.cpp:104-106), resident in HBM.
struct SetDev {
    const int8_t* frag;    // 127 - d as i8, "fragment-major" tiles: [tile][u 0..1][kstep 0..3][lane 0..63][16]
    const int* norm;       // per tile kNormWords: floor(n2/2), n2 & 1, c, early-phase key addends (knn.hip prep_tile)
    const float* f32;      // row-major n x 128 fp32 (the caller's CV_32F rows)
    const float2* kp;      // KeyPoint::pt per row
    int n;
    int n_tiles;           // ceil(n / 64)
    int* flags;            // bit0: a value is not an integer in [0,255]
};

// Deferred prep of one set (i8 fragments, norms, integrality flag), batched per match call.
struct PrepJob {
    const float* src;
    int8_t* frag;
    int* norm;
    int* flags;
    int n;
    int tile0;  // first block of this set in the batched launch
};

struct Top2 {  // partial top-2 of one query over one train split; key = distance (float)
    float k1; int i1; float k2; int i2;
};

// Per-problem device record (knn + ratio + RANSAC).  Built by the host launcher.
struct ProbDev {
    SetDev q, t;
    int nsplit;          // train splits for the distance kernel
    int q_pad;           // nq rounded up to kKnnBlockQ
    long long part_off;  // into Top2 partials: [split][q_pad]
    long long good_off;  // into good arrays (capacity nq)
    long long it_off;    // into per-iteration arrays (capacity max_iters)
};

// Segment of the distance kernel: kKnnBlockQ queries x a train tile range of one problem, written
// to train split `split`.  A block runs the segments seg_start[b] .. seg_start[b + 1] - 1 (api.cpp
// build_tables: one balanced chunk of the batch's tiles per resident block).
struct KnnWork {
    int problem;
    int q0;        // first query row (multiple of kKnnBlockQ)
    int tile0;     // train tiles [tile0, tile1)
    int tile1;
    int split;
};

// RANSAC state per problem (RANSACPointSetRegistrator::run locals, ptsetreg.cpp).
struct RansacState {
    long long stream_pos;  // RNG draws consumed so far (all calls see RNG((uint64)-1))
    int produced;          // samples produced (iterations whose getSubset succeeded)
    int fail_iter;         // iteration whose getSubset failed after 10000 attempts (-1: none)
    int fail_run;          // consecutive failed subset attempts carried across sampler rounds
    int niters;            // current iteration bound (RANSACUpdateNumIters)
    int max_good;          // maxGoodCount
    int best_iter;         // iteration of bestModel
    int next_iter;         // first iteration not yet replayed by the select kernel
    int done;              // loop finished (iter >= niters or getSubset failure)
    int n;                 // point count (= n_good)
    int active;            // problem takes the RANSAC path (n_good > 4)
    int lo_max;            // max lower-bound count seen (filtered path: lower bound of maxGoodCount)
    unsigned long long modM;  // Lemire fast-modulo constant for % n (RNG::uniform(0, n))
    long long win_base;    // stream position of flags[0] of the current chunk's attempt window
    int win_len;           // attempts precomputed in that window
    float sa, sb;          // power-of-two scales of the source / destination coordinates (MFMA bound)
    float smax;            // max over points of |x|+|y|+|u|+|v| (MFMA bound margin)
    int defer;             // chunk 1's exact pass deferred to chunk 2's (no early stop possible in chunk 1)
};

struct RansacParams {
    double thresh;   // reprojection threshold (5.0)
    double conf;     // 0.995
    int max_iters;   // 2000 (reference) / 50000 (BASELINE C3/C4)
    float ratio;
    int min_good, min_inliers;
    double det_lo, det_hi;
    int cand_cap;    // candidate-list capacity per problem and chunk (0: kCandPerProblem)
    int rep_cap;     // attempt kernel's list of repeated-index positions per block (0: kAttemptRepCap)
};

}  // namespace mim

namespace mim {
constexpr int kCandPerProblem = 1024;  // listed exact-evaluation candidates per problem and chunk
constexpr int kIrrBlock = 16384;       // attempt positions per irregular-list block
constexpr int kRansacDefSlots = 16;             // deferred attempts listed per check round (ransac.hip)
#ifndef MIM_CHECK_PER
#define MIM_CHECK_PER 4  // chain attempts per thread and check round (ransac.hip kCheckPer)
#endif
constexpr int kRansacDefRoundAttempts = 256 * MIM_CHECK_PER;  // chain attempts per check round (kCheckBlock x kCheckPer)
constexpr int kIrrCap = 4096;          // listed irregular attempts per block (25 %: n >= ~25 points fit)

// Device buffers of one RANSAC batch (owned by the ctx in api.cpp).
struct RansacBufs {
    RansacState* state;       // [n_probs]
    int4* samples;            // [it_off + iter]  4 point indices of the minimal sample
    float* hyp;               // [(it_off + iter) * 8]  (float)H[0..7] of the minimal-sample model
    int* counts;              // [it_off + iter]  inlier count, -1 when runKernel returned 0
    int2* bounds;             // [it_off + iter]  (lower, upper) bound of the count (filtered path)
    double* best_h;           // [problem][9] bestModel of the filtered select (double H of the best sample)
    int* cand;                // [problem][list 0..1][kCandPerProblem] candidate iterations (list = chunk)
    int* ncand;               // [problem][list] candidates listed (may exceed the capacity)
    int* cex;                 // [problem][list][kCandPerProblem] their exact inlier counts
    double* cH;               // [problem][list][kCandPerProblem][9] their exact models
    int* decided;             // [problem][list][kCandPerProblem] 1: the prescreen decided the listed candidate
    uint8_t* flags;           // [problem][window] getSubset attempt outcomes ahead of stream_pos (written and
                              // valid only where irr_bits is set: the repeated-index and serial attempts)
    uint8_t* irr_bits;        // [problem][window / 8] bit per attempt position: irregular (its flag byte is
                              // written); a clear bit means kPassUnknown (4 draws, checkSubset not evaluated)
    long long flag_cap;       // bytes of `flags`
    int* irr;                 // [problem][block][kIrrCap] positions of irregular attempts (chain sampler)
    int* irr_cnt;             // [problem][block] their count (-1: more than kIrrCap)
    uint32_t* pass_bits;      // [problem][window / 32] bit per chain attempt: checkSubset passes
    void* chains;             // [problem] ChainSegs (ransac.hip): the walked chain of the chunk
    int2* defer;              // [problem][check round][kDefSlots] deferred attempts (attempt index, position)
    int* defer_n;             // [problem][check round] how many are listed
    int def_rounds;           // check rounds per problem with a list (0: every deferred attempt in place)
    int irr_blocks;           // list blocks per problem
    const uint32_t* stream;   // raw cv::RNG((uint64)-1).next() stream shared by every problem
    long long stream_len;
    float4* inl;              // [good_off + k] compressed inliers for the refit (scratch)
    uint4* tiles;             // [good_off / 32 + tile][2][64] f16 MFMA operand tiles of the points
    int* err;                 // device error word (bit0: RNG stream exhausted)
    // Sampler stream: the getSubset replay of chunk c+1 runs on s2 concurrently with the bound /
    // candidate / exact / replay kernels of chunk c (null: everything on the caller's stream)
    hipStream_t s2;
    hipEvent_t ev_fork;
    hipEvent_t ev_samp[2];
};
}  // namespace mim

// SIFT detectAndCompute + 8-bit linear resize (sift.hip), driven by mim_sift_detect_compute /
// mim_resize_linear_u8 (api.cpp).  Return 0, -1 on a HIP error, -2 when the caller's keypoint buffer is
// too small (the counts are set), -3 on a bad argument, -4 when an internal hard limit is exceeded
// (image size, candidates, keypoints, Gaussian kernel size); `err` gets the text.
#include <string>
#include <vector>
#include "../../include/mim.h"
namespace mim {
struct SiftWs;
SiftWs* sift_ws_create();
void sift_ws_destroy(SiftWs* w);
int sift_detect_compute(SiftWs* w, hipStream_t st, const uint8_t* img, int rows, int cols, long long step,
                        const uint8_t* mask, long long mstep, int max_kp, mim_keypoint* kps, float* desc, int* n_out,
                        std::string& err);
int sift_detect_compute_scales(std::vector<SiftWs*>& ws, hipStream_t st, const uint8_t* img, int rows, int cols,
                               long long step, int n_scales, const float* scales, int max_kp, mim_keypoint* kps,
                               float* desc, int* n_out, std::string& err);
int sift_resize_u8(SiftWs* w, hipStream_t st, const uint8_t* src, int rows, int cols, long long step, uint8_t* dst,
                   int drows, int dcols, double fx, double fy, std::string& err);
// the keypoints / descriptors of one image left on the device by sift_scales_device
struct SiftDevOut {
    const mim_keypoint* kp;
    const float* desc;
    int n;
};
int sift_scales_device(std::vector<SiftWs*>& ws, hipStream_t st, const uint8_t* img, int rows, int cols,
                       long long step, int n_scales, const float* scales, SiftDevOut* out, std::string& err);
// out[j]'s n rows and keypoint positions into ddesc[j] / dkp[j], j < n <= 8, one launch (0, -1 HIP error)
int sift_copy_sets(const SiftDevOut* out, int n, float* const* ddesc, float2* const* dkp, hipStream_t st);
}  // namespace mim
