// Test driver for include/mim_detect.hpp (host stages after the matcher, TestsDetector.cpp:112-248,
// utils.cpp:12-20, metrics.cpp:12-186).  tests/test_detect_host.py runs it and checks every output
// against oracle/detect_oracle.py.
//
//   test_detect boxes <points.bin> <out.txt> [results.txt name]
//       points.bin: int32 n, float32 eps, int32 min_points, float32 merge_dist, int32 min_area,
//                   float32 margin_factor, then n x (float32 x, float32 y)
//       out.txt:    the std::unordered_set visiting order, clusters (points as hex floats), discarded
//                   points, per-cluster margin (hex) and box, merged / rejected boxes, detections
//   test_detect metrics <dataset dir> <output dir>
//       mean IoU, per-class IoU and per-class detection accuracy (hex floats)
#include <cstdint>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/mim_detect.hpp"

static void put_pts(FILE* f, const char* tag, const std::vector<mim::Point2f>& v) {
    std::fprintf(f, "%s %zu", tag, v.size());
    for (const auto& p : v) std::fprintf(f, " %a %a", (double)p.x, (double)p.y);
    std::fprintf(f, "\n");
}

static void put_box(FILE* f, const char* tag, const mim::Rect& b) {
    std::fprintf(f, "%s %d %d %d %d\n", tag, b.x, b.y, b.width, b.height);
}

static int boxes(int argc, char** argv) {
    std::ifstream in(argv[2], std::ios::binary);
    int32_t n = 0, min_pts = 0, min_area = 0;
    float eps = 0, merge = 0, factor = 0;
    in.read((char*)&n, 4);
    in.read((char*)&eps, 4);
    in.read((char*)&min_pts, 4);
    in.read((char*)&merge, 4);
    in.read((char*)&min_area, 4);
    in.read((char*)&factor, 4);
    std::vector<mim::Point2f> pts((size_t)n);
    in.read((char*)pts.data(), (std::streamsize)n * 8);
    if (!in) return 2;
    mim::BoxParams bp;
    bp.cluster_distance = eps;
    bp.min_points_per_cluster = min_pts;
    bp.box_merge_distance = merge;
    bp.min_box_area = min_area;
    bp.dynamic_margin = factor;
    mim::Detections dets;
    const std::string name = argc > 5 ? argv[5] : "object";
    const mim::ModelBoxes r = mim::boxes_for_model(pts, name, dets, bp);
    FILE* f = std::fopen(argv[3], "w");
    if (!f) return 3;
    {  // the container order the reference's BFS visits (std::unordered_set<size_t> of 0..n-1)
        std::unordered_set<size_t> s;
        for (size_t i = 0; i < (size_t)n; ++i) s.insert(i);
        std::fprintf(f, "order %d", n);
        for (size_t i : s) std::fprintf(f, " %zu", i);
        std::fprintf(f, "\n");
    }
    for (size_t c = 0; c < r.clusters.kept.size(); ++c) {
        put_pts(f, "cluster", r.clusters.kept[c]);
        std::fprintf(f, "margin %a\n", (double)mim::cluster_margin(r.clusters.kept[c], factor));
        put_box(f, "clusterbox", r.cluster_boxes[c]);
    }
    put_pts(f, "discarded", r.clusters.discarded);
    for (const auto& b : r.merged) put_box(f, "merged", b);
    for (const auto& b : r.rejected) put_box(f, "rejected", b);
    for (const auto& d : dets) put_box(f, "det", d.first);
    std::fclose(f);
    if (argc > 4 && !mim::save_detections(argv[4], dets)) return 4;
    return 0;
}

static int metrics(char** argv) {
    const float miou = mim::compute_mean_intersection_over_union(argv[2], argv[3]);
    std::printf("mean_iou %a\n", (double)miou);
    std::vector<std::string> classes;
    for (const auto& e : std::filesystem::directory_iterator(argv[2]))
        if (e.is_directory()) classes.push_back(e.path().filename().string());
    for (const auto& c : classes)
        std::printf("class_iou %s %a\n", c.c_str(),
                    (double)mim::compute_intersection_over_union(std::string(argv[2]) + "/" + c + "/labels",
                                                                 std::string(argv[3]) + "/" + c));
    for (const auto& [cls, acc] : mim::compute_detection_accuracy(argv[2], argv[3]))
        std::printf("accuracy %s %a\n", cls.c_str(), (double)acc);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 4 && std::string(argv[1]) == "boxes") return boxes(argc, argv);
    if (argc >= 4 && std::string(argv[1]) == "metrics") return metrics(argv);
    std::fprintf(stderr, "usage: test_detect boxes <points.bin> <out.txt> [results.txt name] | metrics <dataset> <output>\n");
    return 1;
}
