// The several-GPU group of include/mim.h through the C ABI (mim_group_*), against one ctx.
//
// A scene batch run by a group must give exactly the records mim_batch_run gives for the same
// problems on one ctx (TestsDetector.cpp:58-95 per scene, Output.cpp:23-57 over the scenes): byte for
// byte, in scene-major, template order.  On a one-GPU box the group is built on device 0 alone (RCCL
// all-gather, a one-rank communicator) and with device 0 repeated (2 and 3 ranks: the copy gather),
// with scene counts that do not divide evenly, and twice on one group (the scene sets replaced).
// Prints "OK group" on success.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/mim.h"

namespace {

struct Lcg {
    unsigned long long s;
    explicit Lcg(unsigned long long seed) : s(seed) {}
    unsigned next() {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        return (unsigned)(s >> 33);
    }
    float uni() { return (next() & 0xFFFFFF) / float(1 << 24); }
};

struct Set {
    std::vector<float> desc, kp;
    int n = 0;
};

// SIFT-like integer rows (what the i8 path takes): sparse histogram values in [0, 255]
void random_rows(Lcg& g, int n, std::vector<float>& d) {
    d.resize((size_t)n * 128);
    for (auto& v : d) {
        const unsigned r = g.next() % 100;
        v = r < 40 ? 0.f : (float)(g.next() % (r < 90 ? 40 : 160));
    }
}

Set make_model(Lcg& g, int n) {
    Set s;
    s.n = n;
    random_rows(g, n, s.desc);
    s.kp.resize((size_t)n * 2);
    for (int i = 0; i < n; ++i) {
        s.kp[2 * i] = 20.f + 600.f * g.uni();
        s.kp[2 * i + 1] = 20.f + 440.f * g.uni();
    }
    return s;
}

// a scene holding `m` noisy copies of model rows under a homography, the rest random
Set make_scene(Lcg& g, const Set& model, int n, int m) {
    Set s;
    s.n = n;
    random_rows(g, n, s.desc);
    s.kp.resize((size_t)n * 2);
    const double a = 0.8 + 0.4 * g.uni(), b = 0.2 * (g.uni() - 0.5), tx = 50 * g.uni(), ty = 40 * g.uni();
    const double p = 1e-4 * (g.uni() - 0.5), q = 1e-4 * (g.uni() - 0.5);
    for (int i = 0; i < n; ++i) {
        if (i < m) {
            const int j = (int)(g.next() % model.n);
            for (int k = 0; k < 128; ++k) {
                float v = model.desc[(size_t)j * 128 + k] + (float)((int)(g.next() % 5) - 2);
                s.desc[(size_t)i * 128 + k] = v < 0 ? 0.f : (v > 255 ? 255.f : v);
            }
            const double x = model.kp[2 * j], y = model.kp[2 * j + 1];
            const double w = p * x + q * y + 1.0;
            s.kp[2 * i] = (float)((a * x + b * y + tx) / w + (g.uni() - 0.5));
            s.kp[2 * i + 1] = (float)((-b * x + a * y + ty) / w + (g.uni() - 0.5));
        } else {
            s.kp[2 * i] = 640.f * g.uni();
            s.kp[2 * i + 1] = 480.f * g.uni();
        }
    }
    return s;
}

int fails = 0;
#define CHECK(cond, ...)                        \
    do {                                        \
        if (!(cond)) {                          \
            printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            printf(__VA_ARGS__);                \
            printf("\n");                       \
            ++fails;                            \
        }                                       \
    } while (0)

// records of the batch on one ctx: views registered first, then every scene's sets in order
std::vector<mim_result> one_ctx(const std::vector<Set>& views, const std::vector<Set>& scenes, int sets_per_scene,
                                const std::vector<mim_problem>& tmpl, const mim_params& prm) {
    mim_ctx* c = nullptr;
    std::vector<mim_result> out;
    if (mim_ctx_create(0, &c) != MIM_OK) {
        CHECK(false, "ctx_create");
        return out;
    }
    int id = 0;
    for (const Set& v : views) mim_set_create(c, v.desc.data(), v.kp.data(), v.n, 128, 0, &id);
    const int base = (int)views.size();
    for (const Set& s : scenes) mim_set_create(c, s.desc.data(), s.kp.data(), s.n, 128, 0, &id);
    const int n_scenes = (int)scenes.size() / sets_per_scene;
    std::vector<mim_problem> probs;
    for (int sc = 0; sc < n_scenes; ++sc)
        for (const mim_problem& t : tmpl) probs.push_back({t.query_set, base + sc * sets_per_scene + t.train_set});
    CHECK(mim_batch_run(c, probs.data(), (int)probs.size(), &prm) == MIM_OK, "batch_run: %s", mim_last_error(c));
    out.resize(probs.size());
    CHECK(mim_batch_results(c, out.data()) == MIM_OK, "batch_results: %s", mim_last_error(c));
    mim_ctx_destroy(c);
    return out;
}

void run_group(const std::vector<int>& devs, const std::vector<Set>& views, const std::vector<std::vector<Set>>& batches,
               int sets_per_scene, const std::vector<mim_problem>& tmpl, const mim_params& prm,
               const std::vector<std::vector<mim_result>>& refs) {
    mim_group* g = nullptr;
    const mim_status cs = mim_group_create(devs.data(), (int)devs.size(), &g);
    CHECK(cs == MIM_OK, "group_create(%zu devices): %d", devs.size(), cs);
    if (cs != MIM_OK) return;
    CHECK(mim_group_size(g) == (int)devs.size(), "group_size");
    for (size_t i = 0; i < views.size(); ++i) {
        int id = -1;
        CHECK(mim_group_set_create(g, views[i].desc.data(), views[i].kp.data(), views[i].n, 128, &id) == MIM_OK,
              "group_set_create: %s", mim_group_last_error(g));
        CHECK(id == (int)i, "replicated set id %d, expected %zu", id, i);
    }
    for (size_t b = 0; b < batches.size(); ++b) {
        const std::vector<Set>& sc = batches[b];
        std::vector<mim_host_set> hs;
        for (const Set& s : sc) hs.push_back({s.desc.data(), s.kp.data(), s.n});
        const int n_scenes = (int)sc.size() / sets_per_scene;
        CHECK(mim_group_scene_batch_run(g, n_scenes, sets_per_scene, hs.data(), (int)tmpl.size(), tmpl.data(), &prm) ==
                  MIM_OK, "scene_batch_run: %s", mim_group_last_error(g));
        std::vector<mim_result> got(refs[b].size());
        CHECK(mim_group_results(g, got.data()) == MIM_OK, "group_results: %s", mim_group_last_error(g));
        int diff = 0;
        for (size_t i = 0; i < got.size(); ++i) diff += memcmp(&got[i], &refs[b][i], sizeof(mim_result)) != 0;
        CHECK(diff == 0, "%zu devices, batch %zu: %d of %zu records differ from one ctx's", devs.size(), b, diff,
              got.size());
        int acc = 0;
        for (const mim_result& r : got) acc += r.status == MIM_ACCEPTED;
        printf("group of %zu (rccl %d) batch %zu: %zu records identical=%d accepted %d\n", devs.size(),
               mim_group_uses_rccl(g), b, got.size(), diff == 0, acc);
    }
    // bad template: a query set that is not replicated
    mim_problem bad{(int)views.size(), 0};
    mim_host_set one{batches[0][0].desc.data(), batches[0][0].kp.data(), batches[0][0].n};
    CHECK(mim_group_scene_batch_run(g, 1, 1, &one, 1, &bad, &prm) == MIM_EINVAL, "bad template accepted");
    mim_group_destroy(g);
}

}  // namespace

int main() {
    Lcg g(0x6A0C1E5ULL);
    std::vector<Set> views = {make_model(g, 700), make_model(g, 500)};
    const int sets_per_scene = 2;
    // the reference's per-scene loop order: model view v at scale k for each (view, scale)
    std::vector<mim_problem> tmpl;
    for (int k = 0; k < sets_per_scene; ++k)
        for (int v = 0; v < 2; ++v) tmpl.push_back({v, k});
    mim_params prm;
    mim_default_params(&prm);
    std::vector<std::vector<Set>> batches(2);
    for (int sc = 0; sc < 7; ++sc)
        for (int k = 0; k < sets_per_scene; ++k)
            batches[0].push_back(make_scene(g, views[(sc + k) % 2], 900 + 37 * sc + 11 * k, 150 + 20 * sc));
    for (int sc = 0; sc < 4; ++sc)
        for (int k = 0; k < sets_per_scene; ++k)
            batches[1].push_back(make_scene(g, views[k], 800 + 13 * sc, sc == 2 ? 3 : 200));  // scene 2: few matches
    std::vector<std::vector<mim_result>> refs;
    for (const auto& b : batches) refs.push_back(one_ctx(views, b, sets_per_scene, tmpl, prm));
    int32_t first = 0, count = 0;
    CHECK(mim_group_shard(7, 3, 2, &first, &count) == MIM_OK && first == 5 && count == 2, "shard");
    run_group({0}, views, batches, sets_per_scene, tmpl, prm, refs);
    run_group({0, 0}, views, batches, sets_per_scene, tmpl, prm, refs);
    run_group({0, 0, 0}, views, batches, sets_per_scene, tmpl, prm, refs);
    if (fails) {
        printf("FAILED %d\n", fails);
        return 1;
    }
    printf("OK group\n");
    return 0;
}
