/*
 * mim.h — C ABI of the MI355X-native matcher + RANSAC homography library (libmim.so).
 *
 * Drop-in boundary for the reference's hot path.  The reference has no plugin/FFI layer: the path
 * is two direct OpenCV calls inside detectObjects (/root/reference/src/TestsDetector.cpp:60,78) plus
 * the glue around them (:62-94).  Each entry point below names the reference interface it replaces.
 * include/mim.hpp is the OpenCV-free C++ layer over this ABI; the cv::Mat-typed drop-in adapter
 * that keeps ObjectModel / processAllModelsImages / detectObjects is adapter/ (built only with
 * OpenCV).
 *
 * Conventions
 *   - POD only, no C++ exceptions cross this boundary; every call returns mim_status.
 *   - Host buffers are owned by the caller.  Device buffers inside a ctx are owned by the ctx.
 *   - One ctx = one GPU + one HIP stream; calls on one ctx are serialised by an internal mutex.
 *   - `_dev`/batch calls are asynchronous on the ctx stream; mim_synchronize() waits.
 *   - Descriptors must be CV_32F rows of dim 128 (SIFT).  Integer-valued rows in [0,255] (what
 *     OpenCV SIFT emits) take the exact-integer i8-MFMA path (v_mfma_i32_32x32x32_i8); any other
 *     rows take the fp32 path in OpenCV's SSE summation order.  Either way indices and distances
 *     are bit-identical to the CPU restatement in oracle/.
 */
#ifndef MIM_H
#define MIM_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct mim_ctx mim_ctx;
typedef int32_t mim_status;
enum {
    MIM_OK = 0,
    MIM_EINVAL = 1,   /* bad argument (null pointer, dim != 128, n < 4 for findHomography, ...) */
    MIM_ENOMODEL = 2, /* findHomography found no model: H.empty() at TestsDetector.cpp:79 */
    MIM_EDEVICE = 3,  /* HIP runtime / RCCL error; text in mim_last_error() */
    MIM_ENOMEM = 4,
    MIM_ERANGE = 5,   /* a capacity was exceeded (e.g. RANSAC RNG stream, the caller's keypoint buffer);
                         text in mim_last_error() */
    MIM_ELIMIT = 6    /* an internal hard limit of the library was exceeded (SIFT: > 16 octaves, > 2^20
                         scale-space candidates, > 2^19 keypoints); retrying with a larger buffer does not
                         help; text in mim_last_error() */
};

/* Problem outcome codes (mim_result.status), TestsDetector.cpp:74-84 */
enum {
    MIM_ACCEPTED = 0,     /* passed every gate: inlier points feed clustering (:87-94) */
    MIM_FEW_GOOD = 1,     /* goodMatches.size() < MIN_INLIERS            (:74) */
    MIM_EMPTY_H = 2,      /* findHomography returned an empty matrix      (:79) */
    MIM_FEW_INLIERS = 3,  /* countNonZero(inlierMask) < MIN_INLIERS       (:81) */
    MIM_BAD_DET = 4,      /* |det H| outside [0.1f, 10.0f]                (:84) */
    MIM_STREAM_SHORT = 5  /* RANSAC needed more RNG draws than the ctx's stream holds: not a result.
                             mim_batch_results / mim_find_homography grow the stream and re-run, so
                             it is only seen in records read on the device (mim_batch_results_dev /
                             _copy) before that */
};

/* Thresholds of detectObjects (TestsDetector.cpp:21-25) + findHomography defaults. */
typedef struct {
    float ratio;          /* MATCH_RATIO_THRESHOLD 0.9f */
    int32_t min_good;     /* MIN_INLIERS 4 (good-match gate, :74) */
    int32_t min_inliers;  /* MIN_INLIERS 4 (inlier gate, :81) */
    double ransac_thresh; /* RANSAC_THRESHOLD 5.0 */
    int32_t max_iters;    /* findHomography maxIters default 2000 */
    double confidence;    /* findHomography confidence default 0.995 */
    double det_lo;        /* (double)0.1f  HOMOGRAPHY_DET_THRESHOLD */
    double det_hi;        /* (double)10.0f HOMOGRAPHY_DET_UPPER_THRESHOLD */
} mim_params;

typedef struct {
    int32_t n_good;   /* ratio-test survivors (goodMatches.size()) */
    int32_t n_inl;    /* countNonZero(inlierMask) */
    int32_t status;   /* MIM_ACCEPTED .. MIM_BAD_DET */
    int32_t iters;    /* RANSAC iterations executed */
    double H[9];      /* row-major, H22 = 1 (zeros when empty) */
    double det;       /* determinant(H) */
} mim_result;

/* One (model view, scene scale) problem: knnMatch(query=view, train=scene) + ratio + RANSAC. */
typedef struct {
    int32_t query_set; /* ObjectModel::descriptors[i] / keypoints[i]  (objectModel.hpp:11-16) */
    int32_t train_set; /* scaled scene descriptors / keypoints         (TestsDetector.cpp:104-106) */
} mim_problem;

const char* mim_version(void);
void mim_default_params(mim_params* p);

mim_status mim_ctx_create(int device, struct mim_ctx** out);
void mim_ctx_destroy(struct mim_ctx* ctx);
const char* mim_last_error(const struct mim_ctx* ctx);
/* Use an external HIP stream (hipStream_t cast to void*); NULL restores the ctx's own stream. */
mim_status mim_ctx_set_stream(struct mim_ctx* ctx, void* stream);
/* Sampler stream on (1) or off (0): with it a batch's second-chunk getSubset replay runs on a second
 * stream of the ctx beside the first chunk's selection kernels (faster for a batch alone); off, one
 * stream (better when several ctxs already overlap their batches).  Default: on, unless the
 * environment has MIM_SAMPLER_STREAM=0.  Takes effect from the next batch. */
mim_status mim_ctx_set_sampler_stream(struct mim_ctx* ctx, int32_t on);
/* The HIP stream the ctx currently enqueues on (its own non-blocking stream unless set above). */
void* mim_ctx_get_stream(const struct mim_ctx* ctx);
mim_status mim_synchronize(struct mim_ctx* ctx);

/* ---- descriptor sets: ObjectModel views and scene scales -------------------------------------
 * Registers n descriptors (n x dim float32, row stride dim) and their keypoints (n x 2 float32,
 * KeyPoint::pt).  on_device == 0: host pointers, copied before the call returns.  on_device != 0:
 * device pointers that the set BORROWS: they are read on the ctx stream by later batch calls (the
 * layout prep, the ratio kernel's keypoint gather, the fp32 and rescan kernels), so they must stay
 * valid and unmodified until mim_sets_clear() / mim_ctx_destroy(), and their producer must be
 * ordered before the ctx stream (the Python Matcher holds the tensors and waits on the producing
 * stream).  The set is converted once into the device layout the kernels stream (DESIGN.md "Data
 * layout in HBM").  Any row count is accepted; a set used as the TRAIN side of a problem must have
 * fewer than 2^18 rows (BFMatcher::knnMatchImpl's assertion), checked at mim_batch_run. */
mim_status mim_set_create(struct mim_ctx* ctx, const float* desc, const float* kp_xy, int32_t n,
                          int32_t dim, int32_t on_device, int32_t* set_id);
/* count sets in one call, as count mim_set_create calls in order (desc[i], kp_xy[i], rows[i]; one
 * on_device flag for all): their ids are *first_id .. *first_id + count - 1.  All or nothing: on an
 * error no set of the call stays registered.  For a caller registering a whole batch of views or
 * scene sets (processAllModelsImages' views, a batch of scenes) without a call per set. */
mim_status mim_sets_create(struct mim_ctx* ctx, int32_t count, const float* const* desc, const float* const* kp_xy,
                           const int32_t* rows, int32_t dim, int32_t on_device, int32_t* first_id);
mim_status mim_sets_clear(struct mim_ctx* ctx);
/* Drops the sets registered after the first n_keep (ids >= n_keep) and reuses their device storage;
 * the first n_keep keep their ids and layout.  The same rules as mim_sets_clear for work already
 * enqueued and borrowed pointers.  For a caller that keeps its model views registered across
 * scenes and replaces only the scene scales (TestsDetector.cpp:38-107 recomputes neither). */
mim_status mim_sets_truncate(struct mim_ctx* ctx, int32_t n_keep);
/* The registered set count and the sets generation: a counter that every mim_sets_clear and every
 * mim_sets_truncate that drops a set increments (never mim_set_create).  A caller that caches set ids
 * across calls (mim.hpp's Detector keeps its model views registered) compares the generation with the
 * one it saw after its own last clear/truncate: a difference means another user of the ctx dropped
 * sets, so the cached ids may name reused storage.  Either output may be NULL. */
mim_status mim_sets_info(struct mim_ctx* ctx, int32_t* n_sets, int64_t* generation);
/* Debug/test copy-out of set `set_id`: its n float32 descriptor rows (n x 128, row-major) and keypoint
 * positions (n x 2) as the kernels read them, e.g. the device-registered scene scales of
 * mim_sift_scales_sets.  Writes min(n, cap) rows (either output may be NULL); *n_rows = n.  Waits for
 * the ctx stream. */
mim_status mim_set_rows(struct mim_ctx* ctx, int32_t set_id, int32_t cap, float* desc, float* kp_xy, int32_t* n_rows);

/* ---- primitive ops, host buffers, synchronous ------------------------------------------------
 * Each primitive call replaces the ctx's "last batch": after mim_knn2_l2 / mim_ratio_filter /
 * mim_knn2_sets_dev there are no records (mim_batch_results returns none), after
 * mim_find_homography there is that call's one record. */
/* ≙ BFMatcher(NORM_L2).knnMatch(q, t, matches, 2)            TestsDetector.cpp:36,60
 * idx[2i+k] = trainIdx of the k-th match of query i (-1 if absent), dist[2i+k] = DMatch::distance. */
mim_status mim_knn2_l2(struct mim_ctx* ctx, const float* q, int32_t nq, const float* t, int32_t nt,
                       int32_t dim, int32_t* idx, float* dist);
/* ≙ the ratio-test loop                                        TestsDetector.cpp:66-72
 * Writes queryIdx/trainIdx of survivors in ascending query order; *n_good = goodMatches.size(). */
mim_status mim_ratio_filter(struct mim_ctx* ctx, const int32_t* idx, const float* dist, int32_t nq,
                            float ratio, int32_t* q_out, int32_t* t_out, int32_t* n_good);
/* ≙ cv::findHomography(src, dst, RANSAC, thresh, mask, max_iters, conf)  TestsDetector.cpp:78
 * src = object points, dst = scene points (n x 2 float32).  mask: n bytes.  Returns MIM_ENOMODEL
 * (H zeroed, mask zeroed) when OpenCV would return an empty Mat; MIM_EINVAL for n < 4. */
mim_status mim_find_homography(struct mim_ctx* ctx, const float* src_xy, const float* dst_xy,
                               int32_t n, double thresh, int32_t max_iters, double conf,
                               double H[9], uint8_t* mask);

/* ---- fused batched path (the detectAtScale view loop, TestsDetector.cpp:58-95) ---------------
 * Enqueues knn2 + ratio + RANSAC + refine + gates for n problems on the ctx stream; returns
 * without waiting.  Results stay on the device until fetched. */
mim_status mim_batch_run(struct mim_ctx* ctx, const mim_problem* problems, int32_t n,
                         const mim_params* params);
/* Waits, then copies the n mim_result records to host memory.  A problem that ran out of RNG
 * draws (MIM_STREAM_SHORT) makes the ctx grow its stream (x8, up to 2^30 draws) and re-run the
 * batch first; that needs the batch's sets intact (no mim_sets_clear since mim_batch_run), else
 * MIM_ERANGE. */
mim_status mim_batch_results(struct mim_ctx* ctx, mim_result* out);
/* Device pointer to the n mim_result records of the last batch (valid until the next batch). */
const mim_result* mim_batch_results_dev(struct mim_ctx* ctx);
/* Copies the n records of the last batch into dst (device memory when dst_on_device != 0: async on
 * the ctx stream, for an RCCL gather; host memory otherwise: synchronous, as mim_batch_results).
 * The device copy does not wait, so it cannot grow the stream and re-run: a record whose status is
 * MIM_STREAM_SHORT is a problem cut short, and the caller re-runs the batch through
 * mim_batch_results (bench.py counts such records as stream_short). */
mim_status mim_batch_results_copy(struct mim_ctx* ctx, void* dst, int32_t dst_on_device);
/* Waits, then copies problem i's good matches (n_good query/train indices, ascending query order)
 * and its RANSAC inlier mask (n_good bytes).  Any output may be NULL. */
mim_status mim_batch_problem_detail(struct mim_ctx* ctx, int32_t i, int32_t* q_idx, int32_t* t_idx,
                                    uint8_t* mask);
/* allUnfilteredScenePts of the last batch, gathered on the device (TestsDetector.cpp:87-94): for every
 * accepted problem (MIM_ACCEPTED) in batch order, the scene keypoints of its RANSAC inliers in mask
 * order, each divided by scales[i] in float when scales[i] != 1.0f (scalePoints, :48-55; scales NULL:
 * no division).  offsets (n + 1 entries): problem i's points are out_xy[2 offsets[i] .. 2 offsets[i+1]);
 * rejected problems have none, so a model whose problems are contiguous in the batch gets its points
 * as one slice.  Waits for the batch (re-running it if the RNG stream was short, as
 * mim_batch_results), then one table copy in, one kernel, one copy out — instead of a
 * mim_batch_problem_detail round trip per accepted problem.  out_xy NULL: offsets only;
 * offsets[n] > cap: MIM_ERANGE (offsets valid, nothing copied).  MIM_EINVAL if the sets were cleared or
 * truncated (mim_sets_clear / mim_sets_truncate) after mim_batch_run: the points are read from them;
 * MIM_EINVAL too after mim_find_homography, whose one record has no scene set to gather from (use
 * its mask with the caller's own points). */
mim_status mim_batch_inlier_points(struct mim_ctx* ctx, const float* scales, float* out_xy, int64_t cap,
                                   int64_t* offsets);

/* ---- distance kernel alone on registered sets (C5 dense-contraction config) ------------------
 * Asynchronous.  idx_dev / dist_dev: device buffers of 2*nq int32 / float32. */
mim_status mim_knn2_sets_dev(struct mim_ctx* ctx, int32_t query_set, int32_t train_set,
                             int32_t* idx_dev, float* dist_dev);

/* ---- feature extraction either side of the matcher ---------------------------
 * cv::KeyPoint without class_id; octave packed as OpenCV packs it (octave & 255 | layer << 8 |
 * sub-layer << 16, octave -1 for the doubled image). */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave;
} mim_keypoint;

/* SIFT::create()->detectAndCompute(gray, mask, kps, desc) with the reference's defaults
 * (main.cpp:17; called at ModelsDetector.cpp:75 with the model mask and at TestsDetector.cpp:106
 * with an empty mask).  gray: host CV_8UC1 rows x cols, row stride `step` bytes; mask: NULL or host
 * CV_8UC1 of the same size, stride mask_step.  Writes min(found, max_kp) keypoints (OpenCV's order:
 * KeypointGreater after removeDuplicatedSorted, then the mask filter) and their 128-float
 * descriptors (row-major); *n_kp = keypoints found (may exceed max_kp: MIM_OK, call again with room
 * for all).  MIM_ELIMIT past the library's hard limits (nothing written).  Synchronous. */
mim_status mim_sift_detect_compute(struct mim_ctx* ctx, const uint8_t* gray, int32_t rows, int32_t cols,
                                   int64_t step, const uint8_t* mask, int64_t mask_step, int32_t max_kp,
                                   mim_keypoint* kps, float* desc, int32_t* n_kp);
/* TestsDetector.cpp:99-107 for one scene in one call: for each of the n_scales scales s,
 * resize(scene, scaled, Size(), s, s, INTER_LINEAR) then SIFT detectAndCompute(scaled) — the scene
 * uploaded once, the resizes on the device, the stages of all scales enqueued together (4 host
 * synchronisations in all instead of 3 per image plus one per resize).  Results are those of
 * mim_resize_linear_u8 + mim_sift_detect_compute per scale: keypoints / descriptors concatenated in
 * scale order into kps / desc (max_kp rows in all), n_kp[s] = keypoints of scale s.  More than max_kp
 * in all: MIM_ERANGE with the counts set (only the first max_kp written); MIM_ELIMIT as above. */
mim_status mim_sift_detect_compute_scales(struct mim_ctx* ctx, const uint8_t* gray, int32_t rows, int32_t cols,
                                          int64_t step, int32_t n_scales, const float* scales, int32_t max_kp,
                                          mim_keypoint* kps, float* desc, int32_t* n_kp);

/* TestsDetector.cpp:99-107 with the results left on the device: resize + SIFT at every scale exactly as
 * mim_sift_detect_compute_scales (n_scales <= 8), then each scale's descriptors and keypoint positions
 * registered as a set of this ctx (as mim_set_create would, but copied on the device: no descriptor
 * leaves the GPU).  set_ids[s] = the set of scale s, n_kp[s] its keypoints.  kps (nullable; max_kp
 * rows) receives the keypoints concatenated in scale order; more than max_kp: MIM_ERANGE after the
 * sets were registered (only the first max_kp written).  One host synchronisation (the counts), two
 * with kps.  The sets follow the rules of mim_set_create (dropped by mim_sets_clear / _truncate). */
mim_status mim_sift_scales_sets(struct mim_ctx* ctx, const uint8_t* gray, int32_t rows, int32_t cols, int64_t step,
                                int32_t n_scales, const float* scales, int32_t* set_ids, int32_t* n_kp, int32_t max_kp,
                                mim_keypoint* kps);

/* cv::resize(src, dst, dsize, fx, fy, INTER_LINEAR) of a CV_8UC1 image (TestsDetector.cpp:102, the
 * scene scales).  fx, fy > 0: resize(src, dst, Size(), fx, fy) — the caller passes
 * drows = cvRound(rows * fy), dcols = cvRound(cols * fx) and OpenCV's coefficients use 1/fx, 1/fy;
 * fx = fy = 0: dsize given.  src stride `step` bytes, dst dense drows x dcols.  Synchronous. */
mim_status mim_resize_linear_u8(struct mim_ctx* ctx, const uint8_t* src, int32_t rows, int32_t cols, int64_t step,
                                uint8_t* dst, int32_t drows, int32_t dcols, double fx, double fy);

/* ---- host stage after the matcher: clustering, margins, merge, area gate (TestsDetector.cpp:111-248)
 * Host code (include/mim_detect.hpp), no ctx, no device.  Thresholds: TestsDetector.cpp:26-30. */
typedef struct {
    float cluster_distance;          /* CLUSTER_DISTANCE_THRESHOLD 20.0f */
    int32_t min_points_per_cluster;  /* MIN_POINTS_PER_CLUSTER 18 */
    float box_merge_distance;        /* BOX_MERGE_DISTANCE 250.0f */
    int32_t min_box_area;            /* MIN_BOX_AREA 2500 */
    float dynamic_margin;            /* DYNAMIC_MARGIN 1.0f */
} mim_box_params;

typedef struct {
    int32_t x, y, width, height; /* cv::Rect */
} mim_rect;

void mim_default_box_params(mim_box_params* p);
/* One model's boxes from its allUnfilteredScenePts (n x 2 float32, the inlier scene points of every
 * accepted (view, scale) problem in the reference's order): writes the merged boxes that pass the
 * area gate, in the reference's order, at most `cap` of them; *n_boxes = their number. */
mim_status mim_detect_boxes(const float* pts_xy, int32_t n, const mim_box_params* bp, mim_rect* boxes, int32_t cap,
                            int32_t* n_boxes);

/* ---- several GPUs of one node: scene-batch data parallelism ------------------
 * Replaces the reference's one-GPU-less loop over the test scenes (processAllTestImages,
 * Output.cpp:23-57, each scene into detectObjects, TestsDetector.cpp:58-95) for one process that owns
 * every GPU of the node.  A group = one ctx per device + an RCCL communicator over them
 * (ncclCommInitAll).  Query (model view) sets are replicated: mim_group_set_create registers the same
 * host set on every device, with the same id.  A scene batch is split into contiguous scene ranges
 * (mim_group_shard: sizes differ by at most one); each device uploads only its own scenes' sets and
 * runs its problems as one mim_batch_run on its ctx; then ONE ncclAllGather over xGMI puts every
 * device's mim_result records (padded to the largest range) on every device.  No descriptor crosses
 * devices.  A device list that repeats a device (two ctxs on one GPU, for tests on a one-GPU machine)
 * gathers with device-to-device copies instead of RCCL (mim_group_uses_rccl() == 0). */
typedef struct mim_group mim_group;
/* One scene set in host memory (n x 128 float32 descriptors, n x 2 float32 keypoint positions). */
typedef struct {
    const float* desc;
    const float* kp_xy;
    int32_t n;
} mim_host_set;

/* ≙ shard.shard_range: rank's contiguous share [*first, *first + *count) of n_items.  No device. */
mim_status mim_group_shard(int32_t n_items, int32_t world, int32_t rank, int32_t* first, int32_t* count);
mim_status mim_group_create(const int32_t* devices, int32_t n_devices, mim_group** out);
void mim_group_destroy(mim_group* g);
int32_t mim_group_size(const mim_group* g);
int32_t mim_group_uses_rccl(const mim_group* g);
/* The ctx of rank r (its device's), for per-device calls (timing, streams); owned by the group. */
struct mim_ctx* mim_group_ctx(mim_group* g, int32_t rank);
const char* mim_group_last_error(const mim_group* g);
/* ObjectModel view registered on every device (host buffers, copied); same id on every ctx.  Drops
 * the scene sets of the last batch.  All or nothing. */
mim_status mim_group_set_create(mim_group* g, const float* desc, const float* kp_xy, int32_t n, int32_t dim,
                                int32_t* set_id);
/* Enqueues a batch of n_scenes scenes.  Scene s owns scene_sets[s * sets_per_scene ..
 * (s + 1) * sets_per_scene) (its scales, host memory, read before the call returns).  Every scene runs
 * the same problem template tmpl[0 .. n_tmpl): query_set = a replicated set id, train_set = an index
 * 0 .. sets_per_scene - 1 into the scene's own sets (the reference's per-scene (model, scale, view)
 * loop: TestsDetector.cpp:38,100,58).  Records: n_scenes * n_tmpl, scene-major, template order within
 * a scene — exactly the records mim_batch_run gives for the same problems on one device.  Returns once
 * every device's batch and the all-gather are enqueued. */
mim_status mim_group_scene_batch_run(mim_group* g, int32_t n_scenes, int32_t sets_per_scene,
                                     const mim_host_set* scene_sets, int32_t n_tmpl, const mim_problem* tmpl,
                                     const mim_params* params);
/* Waits for the batch and its gather; copies the n_scenes * n_tmpl records (from device 0's gathered
 * buffer) to `out` (NULL: wait only).  A device whose problems ran out of RNG draws grows its stream
 * and re-runs its share first, as mim_batch_results. */
mim_status mim_group_results(mim_group* g, mim_result* out);

/* ---- introspection for benches / profiles ----------------------------------------------------- */
/* Per-kernel device time (ms) summed over the batches since the last result fetch, measured with
 * HIP events on the stream each kernel ran on.  names: "knn", "ratio", "attempt", "chain",
 * "check", "sample", "score" (the bound kernel; "hypo"/"score"/"select" in the MIM_RANSAC_EXACT
 * reference mode), "cand", "exact", "select" (the replay), "refine".  Returns -1 if unknown. */
double mim_last_kernel_ms(struct mim_ctx* ctx, const char* name);
mim_status mim_set_timing(struct mim_ctx* ctx, int32_t enable);

#ifdef __cplusplus
}
#endif
#endif
