// The C++ drop-in path on the reference's own images (tests/test_cpp_host.py writes them as raw files):
// ModelsDetector.cpp:46-80 for one object — Detector::sift(view, mask) per view — then, per scene,
// TestsDetector.cpp:32-251 — Detector::detect_scene_gray (resize + SIFT of the five scales on the device,
// every (scale, view) problem in one batch) and mim::boxes_for_model (mim_detect.hpp).  Writes each
// scene's allUnfilteredScenePts (float32 x, y) and detections (int32 x, y, w, h) for the test to compare
// with the golden outputs of the restatement (tests/golden/c1_sugar_box.npz).
//
// usage: detector_real <dir> <rows> <cols> <n_views> <scene>...   (dir holds view_<i>.u8, mask_<i>.u8,
//        scene_<name>.u8; writes pts_<name>.f32 and boxes_<name>.i32)
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "mim.hpp"
#include "mim_detect.hpp"

static std::vector<uint8_t> read_raw(const std::string& path, size_t n) {
    std::ifstream f(path, std::ios::binary);
    std::vector<uint8_t> v((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (v.size() != n) {
        std::fprintf(stderr, "bad size %zu for %s\n", v.size(), path.c_str());
        std::exit(2);
    }
    return v;
}

template <class T>
static void write_raw(const std::string& path, const std::vector<T>& v) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
}

int main(int argc, char** argv) {
    if (argc < 6) return 2;
    const std::string dir = argv[1];
    const int rows = std::atoi(argv[2]), cols = std::atoi(argv[3]), nv = std::atoi(argv[4]);
    const size_t px = (size_t)rows * cols;
    try {
        mim::Detector det(0);
        mim::ModelViews model;
        model.name = "004_sugar_box";
        for (int i = 0; i < nv; ++i) {
            const auto gray = read_raw(dir + "/view_" + std::to_string(i) + ".u8", px);
            const auto mask = read_raw(dir + "/mask_" + std::to_string(i) + ".u8", px);
            std::vector<mim_keypoint> kps;
            mim::View v;
            det.sift(gray.data(), rows, cols, cols, mask.data(), cols, kps, v.descriptors);
            for (const auto& k : kps) v.keypoints.push_back({k.x, k.y});
            model.views.push_back(std::move(v));
        }
        const std::vector<float> scales = {0.7f, 0.85f, 1.0f, 1.15f, 1.3f};  // TestsDetector.cpp:99
        for (int s = 5; s < argc; ++s) {
            const std::string name = argv[s];
            const auto gray = read_raw(dir + "/scene_" + name + ".u8", px);
            std::vector<std::vector<mim::Point2f>> pts;
            det.detect_scene_gray({&model}, gray.data(), rows, cols, cols, scales, pts);
            std::vector<float> flat;
            for (const auto& p : pts[0]) {
                flat.push_back(p.x);
                flat.push_back(p.y);
            }
            write_raw(dir + "/pts_" + name + ".f32", flat);
            mim::Detections dets;
            mim::boxes_for_model(pts[0], model.name, dets);
            std::vector<int32_t> boxes;
            for (const auto& d : dets) {
                boxes.push_back(d.first.x);
                boxes.push_back(d.first.y);
                boxes.push_back(d.first.width);
                boxes.push_back(d.first.height);
            }
            write_raw(dir + "/boxes_" + name + ".i32", boxes);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "FAIL %s\n", e.what());
        return 1;
    }
    std::printf("OK\n");
    return 0;
}
