// mim.hpp — header-only C++ layer over the C ABI (mim.h) that mirrors the reference's host side.
//
// The reference keeps per-object model views in ObjectModel (/root/reference/include/objectModel.hpp:11-16)
// and runs, for every model and every scene scale, the view loop of detectAtScale
// (/root/reference/src/TestsDetector.cpp:43-96).  This header gives that loop an OpenCV-free form:
//
//   mim::ModelViews  ≙ ObjectModel {name, keypoints[v], descriptors[v]}   (raw float arrays)
//   mim::Detector::detect_at_scale(model, scene_kp, scene_desc, scale, out_pts)
//       ≙ detectAtScale(..., kp, desc, scale): knnMatch + ratio + findHomography + gates per view,
//         appending the inlier scene points divided by `scale` in view order, mask order
//         (TestsDetector.cpp:58-95) — all views of the model as ONE device batch.
//   mim::Detector::detect_scene(models, scales...) — SURVEY §8(f) row 1: every (model, view, scale)
//         problem of a scene in one batch; returns the per-model allUnfilteredScenePts.
//
// With OpenCV present, INTEGRATION.md shows the 20-line patch that swaps the reference's view loop for
// detect_at_scale; the clustering/box code after the loop (TestsDetector.cpp:111-248) is unchanged.
#pragma once
#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "mim.h"
#include "mim_types.hpp"

namespace mim {

// One view of an ObjectModel: n keypoints (KeyPoint::pt) + n x 128 CV_32F descriptors.
struct View {
    std::vector<Point2f> keypoints;
    std::vector<float> descriptors;  // row-major n x 128
    int size() const { return (int)keypoints.size(); }
};

// An object's identity for the Detector's registered-views cache: every constructed, copied, moved or
// assigned-to ModelViews gets a fresh value, so an object that reuses a destroyed one's address (or is
// overwritten by assignment) is never mistaken for it.
class ObjectIdentity {
   public:
    ObjectIdentity() : v_(next()) {}
    ObjectIdentity(const ObjectIdentity&) : v_(next()) {}
    ObjectIdentity& operator=(const ObjectIdentity&) {
        v_ = next();
        return *this;
    }
    uint64_t value() const { return v_; }

   private:
    static uint64_t next() {
        static std::atomic<uint64_t> counter{0};
        return ++counter;
    }
    uint64_t v_;
};

struct ModelViews {
    std::string name;
    std::vector<View> views;  // ObjectModel::descriptors.size() entries
    ObjectIdentity identity{};
};

class Error : public std::runtime_error {
   public:
    Error(mim_status s, const std::string& m) : std::runtime_error(m), status(s) {}
    mim_status status;
};

class Detector {
   public:
    explicit Detector(int device = 0) {
        check(mim_ctx_create(device, &ctx_), "mim_ctx_create");
        mim_default_params(&params_);
    }
    ~Detector() { mim_ctx_destroy(ctx_); }
    Detector(const Detector&) = delete;
    Detector& operator=(const Detector&) = delete;

    mim_params& params() { return params_; }
    mim_ctx* ctx() { return ctx_; }

    // Per-view outcome of the last call (same order as the views).
    const std::vector<mim_result>& last_results() const { return results_; }

    // The model views registered by the last detect_* call are reused while the next call passes the
    // same ModelViews objects (identity, not address: see ObjectIdentity) whose every view has the same
    // descriptor and keypoint storage (pointers and sizes) and the same sampled rows (first, middle and
    // last descriptor row and keypoint), and nobody else has dropped sets of this ctx (mim_sets_info's
    // generation).  A caller that rewrites view contents in place calls this first, so the next call
    // registers them anew: the sampled rows catch most rewrites, not all.
    void invalidate_models() { reg_n_ = -1; }

    // TestsDetector.cpp:58-95 for one model at one scale.
    void detect_at_scale(const ModelViews& model, const std::vector<Point2f>& scene_kp,
                         const std::vector<float>& scene_desc, float scale, std::vector<Point2f>& out_pts) {
        std::vector<std::vector<Point2f>> per_model(1);
        run({&model}, {{&scene_kp, &scene_desc, scale}}, per_model);
        out_pts.insert(out_pts.end(), per_model[0].begin(), per_model[0].end());
    }

    struct ScaledScene {
        const std::vector<Point2f>* kp;
        const std::vector<float>* desc;
        float scale;
    };

    // All (model, scale, view) problems of one scene in one device batch.
    // out[m] receives model m's allUnfilteredScenePts in the reference's order: scales outer,
    // views inner (TestsDetector.cpp:100 wraps :58).
    // TestsDetector.cpp:99-107 and the scene's batch from the grayscale scene itself (CV_8UC1 rows x cols,
    // row stride `step`): resize + SIFT of every scale on the device, the scene's descriptors registered
    // there as sets (mim_sift_scales_sets: they never leave the GPU), then detect_scene's batch.
    void detect_scene_gray(const std::vector<const ModelViews*>& models, const uint8_t* gray, int rows, int cols,
                           int64_t step, const std::vector<float>& scales, std::vector<std::vector<Point2f>>& out) {
        out.assign(models.size(), {});
        register_models(models);
        std::vector<int32_t> ids(scales.size()), n(scales.size());
        check(mim_sift_scales_sets(ctx_, gray, rows, cols, step, (int32_t)scales.size(), scales.data(), ids.data(),
                                   n.data(), 0, nullptr),
              "mim_sift_scales_sets", ctx_);
        run_sets(models, ids, scales, out);
    }

    void detect_scene(const std::vector<const ModelViews*>& models, const std::vector<ScaledScene>& scales,
                      std::vector<std::vector<Point2f>>& out) {
        out.assign(models.size(), {});
        run(models, scales, out);
    }

    // SIFT::create()->detectAndCompute(gray, mask, kps, desc) on the device (ModelsDetector.cpp:75 with
    // the view's mask, TestsDetector.cpp:106 without): keypoints in OpenCV's order + n x 128 CV_32F rows.
    void sift(const uint8_t* gray, int rows, int cols, int64_t step, const uint8_t* mask, int64_t mask_step,
              std::vector<mim_keypoint>& kps, std::vector<float>& desc) {
        int32_t cap = 1 << 14, n = 0;
        for (;;) {
            kps.resize(cap);
            desc.resize((size_t)cap * 128);
            const mim_status s = mim_sift_detect_compute(ctx_, gray, rows, cols, step, mask, mask_step, cap, kps.data(),
                                                         desc.data(), &n);
            check(s, "mim_sift_detect_compute", ctx_);  // MIM_ELIMIT etc. throw: a retry cannot help
            if (n <= cap) break;
            cap = n;  // more keypoints than the buffer (MIM_OK, n > cap): call again with room for all
        }
        kps.resize(n);
        desc.resize((size_t)n * 128);
    }

    // TestsDetector.cpp:99-107 in one call: resize(scene, Size(), s, s) + SIFT for every scale s.
    void sift_scales(const uint8_t* gray, int rows, int cols, int64_t step, const std::vector<float>& scales,
                     std::vector<std::vector<mim_keypoint>>& kps, std::vector<std::vector<float>>& desc) {
        const int ns = (int)scales.size();
        std::vector<int32_t> n(ns, 0);
        std::vector<mim_keypoint> k;
        std::vector<float> d;
        int32_t cap = 1 << 16;
        for (;;) {
            k.resize(cap);
            d.resize((size_t)cap * 128);
            const mim_status s = mim_sift_detect_compute_scales(ctx_, gray, rows, cols, step, ns, scales.data(), cap,
                                                                k.data(), d.data(), n.data());
            if (s == MIM_OK) break;
            int64_t tot = 0;
            for (int32_t x : n) tot += x;
            // retry only for a buffer that was too small; anything else (MIM_ELIMIT, ...) throws
            if (s != MIM_ERANGE || tot <= cap || tot > INT32_MAX) check(s, "mim_sift_detect_compute_scales", ctx_);
            cap = (int32_t)tot;
        }
        kps.assign(ns, {});
        desc.assign(ns, {});
        size_t o = 0;
        for (int i = 0; i < ns; ++i) {
            kps[i].assign(k.begin() + o, k.begin() + o + n[i]);
            desc[i].assign(d.begin() + o * 128, d.begin() + (o + n[i]) * 128);
            o += n[i];
        }
    }

   private:
    static void check(mim_status s, const char* what, mim_ctx* c = nullptr) {
        if (s != MIM_OK) throw Error(s, std::string(what) + ": " + (c ? mim_last_error(c) : "failed"));
    }

    // The model views stay registered across scenes (the models are loaded once, main.cpp:22): a call
    // with the same models (same objects, view counts and descriptor storage) drops only the previous
    // scene's sets (mim_sets_truncate) instead of re-uploading and re-preparing every view.
    void register_models(const std::vector<const ModelViews*>& models) {
        std::vector<RegKey> key;
        for (const ModelViews* m : models) {
            key.push_back({m, m->identity.value(), m->views.size(), nullptr, 0, nullptr, 0, 0});
            for (const View& v : m->views)
                key.push_back({nullptr, 0, 0, v.descriptors.data(), v.descriptors.size(),
                               v.keypoints.empty() ? nullptr : &v.keypoints[0].x, v.keypoints.size(), sample(v)});
        }
        int64_t gen = -1;
        check(mim_sets_info(ctx_, nullptr, &gen), "mim_sets_info", ctx_);
        if (reg_n_ >= 0 && gen == reg_gen_ && key == reg_key_) {
            check(mim_sets_truncate(ctx_, reg_n_), "mim_sets_truncate", ctx_);
            check(mim_sets_info(ctx_, nullptr, &reg_gen_), "mim_sets_info", ctx_);
            return;
        }
        reg_n_ = -1;
        check(mim_sets_clear(ctx_), "mim_sets_clear", ctx_);
        reg_ids_.assign(models.size(), {});
        int32_t n = 0;
        for (size_t m = 0; m < models.size(); ++m)
            for (const View& v : models[m]->views) {
                int32_t id;
                check(mim_set_create(ctx_, v.descriptors.data(), v.keypoints.empty() ? nullptr : &v.keypoints[0].x,
                                     v.size(), 128, 0, &id),
                      "mim_set_create", ctx_);
                reg_ids_[m].push_back(id);
                n = id + 1;
            }
        check(mim_sets_info(ctx_, nullptr, &reg_gen_), "mim_sets_info", ctx_);
        reg_key_ = key;
        reg_n_ = n;
    }

    // FNV-1a over a view's first, middle and last descriptor rows and keypoints
    static uint64_t sample(const View& v) {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&h](const void* p, size_t bytes) {
            const unsigned char* b = (const unsigned char*)p;
            for (size_t i = 0; i < bytes; ++i) h = (h ^ b[i]) * 1099511628211ull;
        };
        const size_t n = v.keypoints.size(), rows = v.descriptors.size() / 128;
        for (size_t r : {size_t(0), rows / 2, rows ? rows - 1 : 0})
            if (r < rows) mix(&v.descriptors[r * 128], 128 * sizeof(float));
        for (size_t r : {size_t(0), n / 2, n ? n - 1 : 0})
            if (r < n) mix(&v.keypoints[r], sizeof(Point2f));
        return h;
    }

    void run(const std::vector<const ModelViews*>& models, const std::vector<ScaledScene>& scales,
             std::vector<std::vector<Point2f>>& out) {
        register_models(models);
        std::vector<int32_t> scene_ids;
        std::vector<float> sv;
        for (const ScaledScene& s : scales) {
            int32_t id;
            check(mim_set_create(ctx_, s.desc->data(), s.kp->empty() ? nullptr : &(*s.kp)[0].x, (int32_t)s.kp->size(),
                                 128, 0, &id),
                  "mim_set_create", ctx_);
            scene_ids.push_back(id);
            sv.push_back(s.scale);
        }
        run_sets(models, scene_ids, sv, out);
    }

    // one batch over every (model, scale, view) problem: the registered views against the scene's sets
    void run_sets(const std::vector<const ModelViews*>& models, const std::vector<int32_t>& scene_ids,
                  const std::vector<float>& scale_of, std::vector<std::vector<Point2f>>& out) {
        const std::vector<std::vector<int32_t>>& view_ids = reg_ids_;
        struct Tag { size_t m, s, v; };
        std::vector<mim_problem> probs;
        std::vector<Tag> tags;
        for (size_t m = 0; m < models.size(); ++m)
            for (size_t s = 0; s < scene_ids.size(); ++s)
                for (size_t v = 0; v < view_ids[m].size(); ++v) {
                    probs.push_back({view_ids[m][v], scene_ids[s]});
                    tags.push_back({m, s, v});
                }
        results_.assign(probs.size(), mim_result{});
        if (probs.empty()) return;
        check(mim_batch_run(ctx_, probs.data(), (int32_t)probs.size(), &params_), "mim_batch_run", ctx_);
        check(mim_batch_results(ctx_, results_.data()), "mim_batch_results", ctx_);
        // :87-94 inlier scene points of the accepted problems (:74, :79, :81, :84), divided by the scale
        // when it is not 1, gathered on the device in batch order (one copy); model m's problems are
        // contiguous in the batch, so its points are one slice
        std::vector<float> sc(probs.size());
        for (size_t i = 0; i < probs.size(); ++i) sc[i] = scale_of[tags[i].s];
        std::vector<int64_t> offs(probs.size() + 1);
        check(mim_batch_inlier_points(ctx_, sc.data(), nullptr, 0, offs.data()), "mim_batch_inlier_points", ctx_);
        std::vector<Point2f> pts((size_t)offs.back());
        if (!pts.empty())
            check(mim_batch_inlier_points(ctx_, sc.data(), &pts[0].x, offs.back(), offs.data()),
                  "mim_batch_inlier_points", ctx_);
        for (size_t i = 0; i < probs.size(); ++i)
            out[tags[i].m].insert(out[tags[i].m].end(), pts.begin() + offs[i], pts.begin() + offs[i + 1]);
    }

    // one entry per model (m, its identity, view count), then one per view (storage and sampled rows)
    struct RegKey {
        const ModelViews* m;
        uint64_t identity;
        size_t n_views;
        const float* desc;
        size_t desc_size;
        const float* kp;
        size_t kp_size;
        uint64_t sampled;
        bool operator==(const RegKey& o) const {
            return m == o.m && identity == o.identity && n_views == o.n_views && desc == o.desc &&
                   desc_size == o.desc_size && kp == o.kp && kp_size == o.kp_size && sampled == o.sampled;
        }
    };
    mim_ctx* ctx_ = nullptr;
    mim_params params_;
    std::vector<mim_result> results_;
    std::vector<RegKey> reg_key_;  // the models whose views are the ctx's first reg_n_ sets
    std::vector<std::vector<int32_t>> reg_ids_;
    int32_t reg_n_ = -1;
    int64_t reg_gen_ = -1;  // the ctx's sets generation after this Detector's last clear/truncate
};

}  // namespace mim
