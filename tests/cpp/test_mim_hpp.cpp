// C++ host-layer test: mim::Detector (include/mim.hpp) vs the CPU restatement running the reference's
// view loop (TestsDetector.cpp:58-95) — identical allUnfilteredScenePts, element for element.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../include/mim.hpp"
#include "../../oracle/mim_oracle.h"

static std::vector<float> sift_like(std::mt19937& g, int n) {
    std::gamma_distribution<double> gam(0.5, 1.0);
    std::vector<float> d((size_t)n * 128);
    for (int i = 0; i < n; ++i) {
        double v[128], nrm = 0;
        for (int k = 0; k < 128; ++k) { v[k] = gam(g); nrm += v[k] * v[k]; }
        nrm = std::sqrt(nrm);
        double n2 = 0;
        for (int k = 0; k < 128; ++k) { v[k] = std::min(v[k] / nrm, 0.2); n2 += v[k] * v[k]; }
        n2 = std::sqrt(n2);
        for (int k = 0; k < 128; ++k) d[(size_t)i * 128 + k] = (float)std::min(255.0, std::rint(v[k] * 512 / n2));
    }
    return d;
}

int main() {
    std::mt19937 g(7);
    std::uniform_real_distribution<float> ux(0, 640), uy(0, 480), un(-0.4f, 0.4f);
    // scene (two scales = two descriptor sets), one model with 3 views planted in both
    const int nt = 1500, nq = 400, plant = 150;
    mim::ModelViews model{"004_sugar_box", {}};
    std::vector<std::vector<mim::Point2f>> skp(2);
    std::vector<std::vector<float>> sdesc(2);
    for (int s = 0; s < 2; ++s) {
        sdesc[s] = sift_like(g, nt);
        for (int i = 0; i < nt; ++i) skp[s].push_back({ux(g), uy(g)});
    }
    for (int v = 0; v < 3; ++v) {
        mim::View view;
        view.descriptors = sift_like(g, nq);
        for (int i = 0; i < nq; ++i) view.keypoints.push_back({ux(g), uy(g)});
        for (int s = 0; s < 2; ++s) {
            const float sc = s == 0 ? 0.85f : 1.0f, tx = 20.f * (v + 1), ty = -10.f * s;
            for (int i = 0; i < plant; ++i) {
                const int row = 100 + v * plant + i;  // disjoint rows per view
                for (int k = 0; k < 128; ++k) sdesc[s][(size_t)row * 128 + k] = view.descriptors[(size_t)i * 128 + k];
                sdesc[s][(size_t)row * 128 + (i % 128)] = std::min(255.f, sdesc[s][(size_t)row * 128 + (i % 128)] + 1.f);
                if (i % 2 == 0) skp[s][row] = {view.keypoints[i].x * sc + tx + un(g), view.keypoints[i].y * sc + ty + un(g)};
            }
        }
        model.views.push_back(std::move(view));
    }
    const float scales[2] = {0.85f, 1.0f};
    mim::Detector det(0);
    det.params().max_iters = 2000;
    std::vector<std::vector<mim::Point2f>> out;
    det.detect_scene({&model}, {{&skp[0], &sdesc[0], scales[0]}, {&skp[1], &sdesc[1], scales[1]}}, out);

    // reference loop on the CPU restatement
    orc_params prm;
    orc_default_params(&prm);
    prm.max_iters = 2000;
    std::vector<mim::Point2f> ref;
    for (int s = 0; s < 2; ++s)
        for (int v = 0; v < 3; ++v) {
            orc_result r;
            std::vector<uint8_t> mask(nq);
            std::vector<int32_t> gq(nq), gt(nq);
            orc_match_problem(model.views[v].descriptors.data(), &model.views[v].keypoints[0].x, nq, sdesc[s].data(),
                              &skp[s][0].x, nt, 128, &prm, 1, &r, mask.data(), gq.data(), gt.data());
            if (r.status != 0) continue;
            for (int j = 0; j < r.n_good; ++j)
                if (mask[j]) {
                    mim::Point2f p = skp[s][gt[j]];
                    if (scales[s] != 1.0f) { p.x /= scales[s]; p.y /= scales[s]; }
                    ref.push_back(p);
                }
        }
    if (out.size() != 1 || out[0].size() != ref.size()) {
        std::printf("FAIL size %zu vs %zu\n", out.empty() ? 0 : out[0].size(), ref.size());
        return 1;
    }
    for (size_t i = 0; i < ref.size(); ++i)
        if (out[0][i].x != ref[i].x || out[0][i].y != ref[i].y) {
            std::printf("FAIL at %zu\n", i);
            return 1;
        }
    // the same scene again: the model's views stay registered (mim_sets_truncate), same points
    std::vector<std::vector<mim::Point2f>> again;
    det.detect_scene({&model}, {{&skp[0], &sdesc[0], scales[0]}, {&skp[1], &sdesc[1], scales[1]}}, again);
    if (again.size() != 1 || again[0].size() != out[0].size()) {
        std::printf("FAIL repeat size\n");
        return 1;
    }
    for (size_t i = 0; i < out[0].size(); ++i)
        if (again[0][i].x != out[0][i].x || again[0][i].y != out[0][i].y) {
            std::printf("FAIL repeat at %zu\n", i);
            return 1;
        }
    // a view rewritten in place (its keypoints moved): after invalidate_models() the next call registers
    // the views anew and equals a fresh Detector's result on the changed model
    {
        for (auto& v : model.views)
            for (auto& k : v.keypoints) k.x += 3.0f;
        det.invalidate_models();
        std::vector<std::vector<mim::Point2f>> moved, fresh;
        det.detect_scene({&model}, {{&skp[0], &sdesc[0], scales[0]}, {&skp[1], &sdesc[1], scales[1]}}, moved);
        mim::Detector det2(0);
        det2.detect_scene({&model}, {{&skp[0], &sdesc[0], scales[0]}, {&skp[1], &sdesc[1], scales[1]}}, fresh);
        bool same = moved.size() == fresh.size() && moved[0].size() == fresh[0].size();
        for (size_t i = 0; same && i < fresh[0].size(); ++i)
            same = moved[0][i].x == fresh[0][i].x && moved[0][i].y == fresh[0][i].y;
        if (!same) {
            std::printf("FAIL invalidate_models\n");
            return 1;
        }
        for (auto& v : model.views)
            for (auto& k : v.keypoints) k.x -= 3.0f;
        det.invalidate_models();
    }
    // the cache without invalidate_models(): (a) a view's descriptors replaced by copy-assignment (the
    // vector keeps its buffer, so only the sampled rows differ), (b) the model overwritten by
    // assignment (fresh identity), (c) the ctx's sets dropped and replaced through det.ctx() (sets
    // generation): each time the result equals a fresh Detector's
    auto same_as_fresh = [&](const mim::ModelViews& mv, const char* what) {
        std::vector<std::vector<mim::Point2f>> a, f;
        det.detect_scene({&mv}, {{&skp[0], &sdesc[0], scales[0]}, {&skp[1], &sdesc[1], scales[1]}}, a);
        mim::Detector det2(0);
        det2.params().max_iters = 2000;
        det2.detect_scene({&mv}, {{&skp[0], &sdesc[0], scales[0]}, {&skp[1], &sdesc[1], scales[1]}}, f);
        bool same = a.size() == f.size() && a[0].size() == f[0].size();
        for (size_t i = 0; same && i < f[0].size(); ++i) same = a[0][i].x == f[0][i].x && a[0][i].y == f[0][i].y;
        if (!same) std::printf("FAIL registered-views cache: %s (%zu vs %zu points)\n", what, a[0].size(), f[0].size());
        return same;
    };
    {
        const std::vector<float> keep1 = model.views[1].descriptors;
        const float* buf = model.views[1].descriptors.data();
        model.views[1].descriptors = model.views[2].descriptors;
        if (model.views[1].descriptors.data() != buf) std::printf("note: the copy-assignment reallocated\n");
        if (!same_as_fresh(model, "view descriptors replaced")) return 1;
        model.views[1].descriptors = keep1;
        if (!same_as_fresh(model, "view descriptors restored")) return 1;
        mim::ModelViews other = model;
        for (auto& k : other.views[0].keypoints) k.y += 2.0f;
        model = other;
        if (!same_as_fresh(model, "model assigned")) return 1;
        for (auto& k : model.views[0].keypoints) k.y -= 2.0f;
        det.invalidate_models();
        if (!same_as_fresh(model, "model restored")) return 1;
        int32_t junk_id = 0;
        if (mim_sets_clear(det.ctx()) != MIM_OK ||
            mim_set_create(det.ctx(), sdesc[0].data(), &skp[0][0].x, nt, 128, 0, &junk_id) != MIM_OK) {
            std::printf("FAIL external sets calls\n");
            return 1;
        }
        if (!same_as_fresh(model, "sets replaced through ctx()")) return 1;
        std::printf("OK registered-views cache\n");
    }
    std::printf("OK %zu inlier points, statuses:", ref.size());
    for (auto& r : det.last_results()) std::printf(" %d/%d/%d", r.n_good, r.n_inl, r.status);
    std::printf("\n");
    if (ref.empty()) return 1;

    // detect_scene_gray (SIFT of the scales left on the device as the batch's sets) equals
    // detect_scene on the host copies of the same SIFT: a smooth synthetic scene and two model views
    // described from crops of it
    const int R = 240, Cc = 320;
    std::vector<uint8_t> img((size_t)R * Cc);
    std::mt19937 g2(3);
    std::uniform_real_distribution<double> ur(0, 1);
    std::vector<double> acc((size_t)R * Cc, 110.0);
    for (int b = 0; b < 60; ++b) {
        const double cy = ur(g2) * R, cx = ur(g2) * Cc, sg = 1.5 + ur(g2) * 18, a = (ur(g2) - 0.5) * 180;
        for (int y = 0; y < R; ++y)
            for (int x = 0; x < Cc; ++x) acc[(size_t)y * Cc + x] += a * std::exp(-((y - cy) * (y - cy) + (x - cx) * (x - cx)) / (2 * sg * sg));
    }
    for (size_t i = 0; i < img.size(); ++i) img[i] = (uint8_t)std::min(255.0, std::max(0.0, std::rint(acc[i] + (ur(g2) - 0.5) * 6)));
    mim::ModelViews crops{"crops", {}};
    for (int v = 0; v < 2; ++v) {
        const int y0 = 20 + 60 * v, x0 = 30 + 90 * v, h = 140, w = 160;
        std::vector<uint8_t> crop((size_t)h * w);
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) crop[(size_t)y * w + x] = img[(size_t)(y0 + y) * Cc + x0 + x];
        std::vector<mim_keypoint> kk;
        mim::View view;
        det.sift(crop.data(), h, w, w, nullptr, 0, kk, view.descriptors);
        for (auto& k : kk) view.keypoints.push_back({k.x, k.y});
        crops.views.push_back(std::move(view));
    }
    const std::vector<float> sc5 = {0.7f, 0.85f, 1.0f, 1.15f, 1.3f};
    std::vector<std::vector<mim_keypoint>> hk;
    std::vector<std::vector<float>> hd;
    det.sift_scales(img.data(), R, Cc, Cc, sc5, hk, hd);
    std::vector<std::vector<mim::Point2f>> hkp(sc5.size());
    std::vector<mim::Detector::ScaledScene> ss;
    for (size_t s = 0; s < sc5.size(); ++s) {
        for (auto& k : hk[s]) hkp[s].push_back({k.x, k.y});
        ss.push_back({&hkp[s], &hd[s], sc5[s]});
    }
    std::vector<std::vector<mim::Point2f>> host_pts, dev_pts;
    det.detect_scene({&crops}, ss, host_pts);
    const std::vector<mim_result> host_res = det.last_results();
    det.detect_scene_gray({&crops}, img.data(), R, Cc, Cc, sc5, dev_pts);
    const std::vector<mim_result>& dev_res = det.last_results();
    if (host_res.size() != dev_res.size() || host_pts[0].size() != dev_pts[0].size()) {
        std::printf("FAIL gray path: %zu/%zu problems, %zu/%zu points\n", host_res.size(), dev_res.size(),
                    host_pts[0].size(), dev_pts[0].size());
        return 1;
    }
    for (size_t i = 0; i < host_res.size(); ++i)
        if (host_res[i].n_good != dev_res[i].n_good || host_res[i].n_inl != dev_res[i].n_inl ||
            host_res[i].status != dev_res[i].status || host_res[i].iters != dev_res[i].iters) {
            std::printf("FAIL gray path record %zu\n", i);
            return 1;
        }
    for (size_t i = 0; i < host_pts[0].size(); ++i)
        if (host_pts[0][i].x != dev_pts[0][i].x || host_pts[0][i].y != dev_pts[0][i].y) {
            std::printf("FAIL gray path point %zu\n", i);
            return 1;
        }
    int accepted = 0;
    for (auto& r : dev_res) accepted += r.status == 0;
    std::printf("OK gray path: %zu problems, %d accepted, %zu points\n", dev_res.size(), accepted, dev_pts[0].size());
    return accepted > 0 ? 0 : 1;
}
