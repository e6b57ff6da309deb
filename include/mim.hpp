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

struct ModelViews {
    std::string name;
    std::vector<View> views;  // ObjectModel::descriptors.size() entries
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
    void detect_scene(const std::vector<const ModelViews*>& models, const std::vector<ScaledScene>& scales,
                      std::vector<std::vector<Point2f>>& out) {
        out.assign(models.size(), {});
        run(models, scales, out);
    }

   private:
    static void check(mim_status s, const char* what, mim_ctx* c = nullptr) {
        if (s != MIM_OK) throw Error(s, std::string(what) + ": " + (c ? mim_last_error(c) : "failed"));
    }

    void run(const std::vector<const ModelViews*>& models, const std::vector<ScaledScene>& scales,
             std::vector<std::vector<Point2f>>& out) {
        check(mim_sets_clear(ctx_), "mim_sets_clear", ctx_);
        std::vector<std::vector<int32_t>> view_ids(models.size());
        for (size_t m = 0; m < models.size(); ++m)
            for (const View& v : models[m]->views) {
                int32_t id;
                check(mim_set_create(ctx_, v.descriptors.data(), v.keypoints.empty() ? nullptr : &v.keypoints[0].x,
                                     v.size(), 128, 0, &id),
                      "mim_set_create", ctx_);
                view_ids[m].push_back(id);
            }
        std::vector<int32_t> scene_ids;
        for (const ScaledScene& s : scales) {
            int32_t id;
            check(mim_set_create(ctx_, s.desc->data(), s.kp->empty() ? nullptr : &(*s.kp)[0].x, (int32_t)s.kp->size(),
                                 128, 0, &id),
                  "mim_set_create", ctx_);
            scene_ids.push_back(id);
        }
        struct Tag { size_t m, s, v; };
        std::vector<mim_problem> probs;
        std::vector<Tag> tags;
        for (size_t m = 0; m < models.size(); ++m)
            for (size_t s = 0; s < scales.size(); ++s)
                for (size_t v = 0; v < view_ids[m].size(); ++v) {
                    probs.push_back({view_ids[m][v], scene_ids[s]});
                    tags.push_back({m, s, v});
                }
        results_.assign(probs.size(), mim_result{});
        if (probs.empty()) return;
        check(mim_batch_run(ctx_, probs.data(), (int32_t)probs.size(), &params_), "mim_batch_run", ctx_);
        check(mim_batch_results(ctx_, results_.data()), "mim_batch_results", ctx_);
        std::vector<int32_t> qi, ti;
        std::vector<uint8_t> mask;
        for (size_t i = 0; i < probs.size(); ++i) {
            const mim_result& r = results_[i];
            if (r.status != MIM_ACCEPTED) continue;  // :74, :79, :81, :84
            qi.resize(r.n_good);
            ti.resize(r.n_good);
            mask.resize(r.n_good);
            check(mim_batch_problem_detail(ctx_, (int32_t)i, qi.data(), ti.data(), mask.data()), "detail", ctx_);
            const ScaledScene& sc = scales[tags[i].s];
            for (int j = 0; j < r.n_good; ++j) {  // :87-94 inlier scene points, /scale when scale != 1
                if (!mask[j]) continue;
                Point2f p = (*sc.kp)[ti[j]];
                if (sc.scale != 1.0f) {
                    p.x /= sc.scale;
                    p.y /= sc.scale;
                }
                out[tags[i].m].push_back(p);
            }
        }
    }

    mim_ctx* ctx_ = nullptr;
    mim_params params_;
    std::vector<mim_result> results_;
};

}  // namespace mim
