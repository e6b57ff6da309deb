// mim_detect.hpp — the host stages after the matcher: inlier clustering, box margin, box merge, area
// gate, results files and the detection metrics.  Header-only C++17, no OpenCV, no device code.
//
// Reference (the code these restate; argument meaning and outputs kept):
//   cluster_points       /root/reference/src/TestsDetector.cpp:112-151  BFS over the inlier scene points,
//                        link if (float)|p - q| <= 20, keep clusters of >= 18 points
//   bounding_rect        cv::boundingRect of CV_32F points (imgproc shapedescr.cpp pointSetBoundingRect)
//   cluster_margin/box   TestsDetector.cpp:154-190  stddev of all pairwise distances, box grown by it
//   merge_boxes          TestsDetector.cpp:193-236  BFS over box centres within 250 px, union rectangle
//   boxes_for_model      TestsDetector.cpp:112-248  the whole stage incl. the area gate (>= 2500)
//   save_detections      src/utils.cpp:12-20        "<name> x0 y0 x1 y1" per line
//   read_boxes_coordinates, iou, compute_*           src/metrics.cpp:12-186
//
// Determinism: the reference keeps the unassigned points in a std::unordered_set<size_t>
// (TestsDetector.cpp:114) and both its "next start" (`*begin()`) and the order in which a point's
// neighbours join the cluster (`for (idx : set)`) follow that container's iteration order.  The
// cluster *sets* do not depend on it, the float sums of the margin (:163-180) do.  cluster_points
// builds the same std::unordered_set once and visits points in its iteration order (erasing never
// reorders the rest of a libstdc++ set), so with the same standard library the point order, and with
// it every margin bit, is the reference's.  The neighbour search is a uniform grid instead of the
// reference's scan of every unassigned point per visited point (O(P) per point instead of O(P^2)
// overall); the pairwise-distance statistics stay the exact sequential float sums (O(P^2) per cluster).
#pragma once
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <filesystem>
#include <fstream>
#include <map>
#include <numeric>
#include <ostream>
#include <queue>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "mim_types.hpp"

namespace mim {

// TestsDetector.cpp:26-30
struct BoxParams {
    float cluster_distance = 20.0f;    // CLUSTER_DISTANCE_THRESHOLD
    int min_points_per_cluster = 18;   // MIN_POINTS_PER_CLUSTER
    float box_merge_distance = 250.0f; // BOX_MERGE_DISTANCE
    int min_box_area = 2500;           // MIN_BOX_AREA
    float dynamic_margin = 1.0f;       // DYNAMIC_MARGIN
};

// cv::norm(Point_<float>) of a float difference: sqrt in double of the float components
inline double point_norm(float dx, float dy) { return std::sqrt((double)dx * dx + (double)dy * dy); }

// the reference's link test (:135): dist = (float)norm(a - b) <= eps, a - b in float
inline bool within(const Point2f& a, const Point2f& b, float eps) {
    return (float)point_norm(a.x - b.x, a.y - b.y) <= eps;
}

struct Clusters {
    std::vector<std::vector<Point2f>> kept;  // pointClusters (:113), in discovery order
    std::vector<Point2f> discarded;          // discardedPtsGlobal (:40, :149)
};

// TestsDetector.cpp:112-151
inline Clusters cluster_points(const std::vector<Point2f>& pts, float eps = 20.0f, int min_points = 18) {
    Clusters out;
    const size_t n = pts.size();
    if (n == 0) return out;
    // visiting order = iteration order of std::unordered_set<size_t>{0..n-1} built by inserting 0..n-1
    std::vector<size_t> order;
    order.reserve(n);
    {
        std::unordered_set<size_t> s;
        for (size_t i = 0; i < n; ++i) s.insert(i);
        order.assign(s.begin(), s.end());
    }
    std::vector<uint32_t> rank(n);
    for (size_t k = 0; k < n; ++k) rank[order[k]] = (uint32_t)k;

    // uniform grid over the finite points (cell a little larger than eps: every float-rounded link
    // lies within the 3x3 block); non-finite points link to nothing (NaN <= eps is false)
    const double cell = (double)eps * (1.0 + 1e-3) + 1e-6;
    auto key = [](int64_t cx, int64_t cy) { return (uint64_t)(cx + (1ll << 31)) << 32 | (uint64_t)(cy + (1ll << 31)); };
    bool grid_ok = eps > 0.f;
    for (const Point2f& p : pts)
        if (std::isfinite(p.x) && std::isfinite(p.y) && (std::fabs(p.x) > 1e9f || std::fabs(p.y) > 1e9f)) grid_ok = false;
    std::unordered_map<uint64_t, std::vector<uint32_t>> grid;
    std::vector<int64_t> cx(n, 0), cy(n, 0);
    std::vector<char> finite(n, 0);
    for (size_t i = 0; i < n; ++i) {
        finite[i] = std::isfinite(pts[i].x) && std::isfinite(pts[i].y);
        if (!finite[i] || !grid_ok) continue;
        cx[i] = (int64_t)std::floor(pts[i].x / cell);
        cy[i] = (int64_t)std::floor(pts[i].y / cell);
        grid[key(cx[i], cy[i])].push_back((uint32_t)i);
    }

    std::vector<char> assigned(n, 0);
    size_t next = 0;  // position in `order` of the first possibly unassigned point (the set's begin())
    std::vector<uint32_t> found;
    for (;;) {
        while (next < n && assigned[order[next]]) ++next;
        if (next == n) break;
        const size_t start = order[next];
        assigned[start] = 1;
        std::vector<Point2f> cur{pts[start]};
        std::queue<size_t> frontier;
        frontier.push(start);
        while (!frontier.empty()) {
            const size_t c = frontier.front();
            frontier.pop();
            found.clear();
            if (finite[c]) {
                if (grid_ok) {
                    for (int64_t dx = -1; dx <= 1; ++dx)
                        for (int64_t dy = -1; dy <= 1; ++dy) {
                            auto it = grid.find(key(cx[c] + dx, cy[c] + dy));
                            if (it == grid.end()) continue;
                            for (uint32_t o : it->second)
                                if (!assigned[o] && within(pts[c], pts[o], eps)) found.push_back(o);
                        }
                } else {
                    for (size_t o = 0; o < n; ++o)
                        if (!assigned[o] && within(pts[c], pts[o], eps)) found.push_back((uint32_t)o);
                }
            }
            // the reference appends them in the set's iteration order, then erases them (:134-143)
            std::sort(found.begin(), found.end(), [&](uint32_t a, uint32_t b) { return rank[a] < rank[b]; });
            for (uint32_t o : found) {
                assigned[o] = 1;
                cur.push_back(pts[o]);
                frontier.push(o);
            }
        }
        if ((int)cur.size() >= min_points) out.kept.push_back(std::move(cur));
        else out.discarded.insert(out.discarded.end(), cur.begin(), cur.end());
    }
    return out;
}

// cv::boundingRect of float points: corners floored, right/bottom exclusive (+1)
inline Rect bounding_rect(const std::vector<Point2f>& pts) {
    if (pts.empty()) return Rect{0, 0, 0, 0};
    float xmin = pts[0].x, xmax = pts[0].x, ymin = pts[0].y, ymax = pts[0].y;
    for (const Point2f& p : pts) {
        xmin = std::min(xmin, p.x);
        xmax = std::max(xmax, p.x);
        ymin = std::min(ymin, p.y);
        ymax = std::max(ymax, p.y);
    }
    const int x0 = (int)std::floor(xmin), y0 = (int)std::floor(ymin);
    const int x1 = (int)std::floor(xmax), y1 = (int)std::floor(ymax);
    return Rect{x0, y0, x1 - x0 + 1, y1 - y0 + 1};
}

// TestsDetector.cpp:160-183: standard deviation of the cluster's pairwise distances (float sums in
// pair order i < j, the squared deviations through double as pow(float, int) promotes) x factor
inline float cluster_margin(const std::vector<Point2f>& c, float factor = 1.0f) {
    std::vector<float> d;
    d.reserve(c.size() * (c.size() - (c.empty() ? 0 : 1)) / 2);
    float mean = 0.0f;
    for (size_t i = 0; i < c.size(); ++i)
        for (size_t j = i + 1; j < c.size(); ++j) {
            const float v = (float)point_norm(c[i].x - c[j].x, c[i].y - c[j].y);
            d.push_back(v);
            mean += v;
        }
    if (!d.empty()) mean /= (float)d.size();
    float var = 0.0f;
    for (float v : d) {
        const float dv = v - mean;
        var += (float)((double)dv * (double)dv);
    }
    return std::sqrt(var / (float)d.size()) * factor;
}

// TestsDetector.cpp:157-187: bounding rectangle grown by the truncated margin on every side
inline Rect cluster_box(const std::vector<Point2f>& c, float factor = 1.0f) {
    Rect b = bounding_rect(c);
    const float m = cluster_margin(c, factor);
    b.x -= (int)m;
    b.y -= (int)m;
    b.width += (int)(2 * m);
    b.height += (int)(2 * m);
    return b;
}

// TestsDetector.cpp:193-236: groups of boxes whose centres chain within max_dist, each replaced by
// the union rectangle; groups in order of their first box
inline std::vector<Rect> merge_boxes(const std::vector<Rect>& boxes, float max_dist = 250.0f) {
    std::vector<Rect> merged;
    std::vector<char> done(boxes.size(), 0);
    auto centre = [&](size_t i) {
        return Point2f{(float)boxes[i].x + (float)boxes[i].width / 2.0f, (float)boxes[i].y + (float)boxes[i].height / 2.0f};
    };
    for (size_t i = 0; i < boxes.size(); ++i) {
        if (done[i]) continue;
        done[i] = 1;
        int x0 = INT_MAX, y0 = INT_MAX, x1 = INT_MIN, y1 = INT_MIN;
        std::queue<size_t> q;
        q.push(i);
        while (!q.empty()) {
            const size_t c = q.front();
            q.pop();
            const Rect& b = boxes[c];
            x0 = std::min(x0, b.x);
            y0 = std::min(y0, b.y);
            x1 = std::max(x1, b.x + b.width);
            y1 = std::max(y1, b.y + b.height);
            const Point2f pc = centre(c);
            for (size_t j = 0; j < boxes.size(); ++j) {
                if (done[j]) continue;
                const Point2f pj = centre(j);
                if (point_norm(pc.x - pj.x, pc.y - pj.y) <= (double)max_dist) {
                    done[j] = 1;
                    q.push(j);
                }
            }
        }
        merged.push_back(Rect{x0, y0, x1 - x0, y1 - y0});
    }
    return merged;
}

using Detections = std::vector<std::pair<Rect, std::string>>;

// What one model contributes, with the intermediate products for inspection/visualisation.
struct ModelBoxes {
    Clusters clusters;
    std::vector<Rect> cluster_boxes;  // clusterBoxes (:155)
    std::vector<Rect> merged;         // mergedBoxes (:193)
    std::vector<Rect> rejected;       // merged boxes below the area gate (:241-246)
};

// TestsDetector.cpp:112-248 for one model: appends (box, name) for every merged box with area >=
// min_box_area to `detections`.  `log` (optional) receives the reference's rejection message.
inline ModelBoxes boxes_for_model(const std::vector<Point2f>& all_scene_pts, const std::string& name,
                                  Detections& detections, const BoxParams& bp = BoxParams(),
                                  std::ostream* log = nullptr) {
    ModelBoxes r;
    if (all_scene_pts.empty()) return r;
    r.clusters = cluster_points(all_scene_pts, bp.cluster_distance, bp.min_points_per_cluster);
    if (r.clusters.kept.empty()) return r;
    for (const auto& c : r.clusters.kept) r.cluster_boxes.push_back(cluster_box(c, bp.dynamic_margin));
    r.merged = merge_boxes(r.cluster_boxes, bp.box_merge_distance);
    for (const Rect& b : r.merged) {
        const int area = b.width * b.height;
        if (area < bp.min_box_area) {
            r.rejected.push_back(b);
            if (log)
                *log << "Rejected box for " << name << " - Area too small: " << area
                     << " (min allowed: " << bp.min_box_area << ")\n";
            continue;
        }
        detections.emplace_back(b, name);
    }
    return r;
}

// src/utils.cpp:12-20: one "<name> x0 y0 x1 y1" line per detection (x1 = x + width, y1 = y + height)
inline bool save_detections(const std::string& path, const Detections& dets) {
    std::ofstream f(path);
    if (!f) return false;
    for (const auto& [b, name] : dets) f << name << " " << b.x << " " << b.y << " " << b.x + b.width << " " << b.y + b.height << "\n";
    return (bool)f;
}

// ---- src/metrics.cpp ------------------------------------------------------------------------------
using BoxMap = std::map<std::string, std::map<std::string, std::vector<int>>>;  // file id -> object id -> box

// metrics.cpp:56-75: every file of the directory, id = file name up to its first '-', lines
// "<object_id> x_min y_min x_max y_max" (a repeated object id keeps the last line)
inline BoxMap read_boxes_coordinates(const std::string& dir) {
    namespace fs = std::filesystem;
    BoxMap boxes;
    for (const fs::directory_entry& e : fs::directory_iterator(dir)) {
        std::ifstream f(e.path());
        const std::string fn = e.path().filename().string();
        const std::string id = fn.substr(0, fn.find('-'));
        std::string obj;
        int a, b, c, d;
        while (f >> obj >> a >> b >> c >> d) boxes[id][obj] = {a, b, c, d};
    }
    return boxes;
}

// metrics.cpp:88-104: integer areas, float ratio (corner boxes x_min y_min x_max y_max)
inline float box_iou(const std::vector<int>& p, const std::vector<int>& q) {
    const int iw = std::max(0, std::min(p[2], q[2]) - std::max(p[0], q[0]));
    const int ih = std::max(0, std::min(p[3], q[3]) - std::max(p[1], q[1]));
    const int inter = iw * ih;
    const int uni = (p[2] - p[0]) * (p[3] - p[1]) + (q[2] - q[0]) * (q[3] - q[1]) - inter;
    return (float)inter / (float)uni;
}

// metrics.cpp:78-86
inline float compute_iou_if_present(const std::string& object_id, const std::vector<int>& gt,
                                    const std::map<std::string, std::vector<int>>& predicted) {
    auto it = predicted.find(object_id);
    return it == predicted.end() ? 0.0f : box_iou(gt, it->second);
}

// metrics.cpp:29-53: mean over every ground-truth object of its IoU (0 when not predicted)
inline float compute_intersection_over_union(const std::string& gt_dir, const std::string& pred_dir,
                                             std::ostream* log = nullptr) {
    const BoxMap gt = read_boxes_coordinates(gt_dir);
    BoxMap pred = read_boxes_coordinates(pred_dir);
    float total = 0.0f;
    int count = 0;
    for (const auto& [file_id, objects] : gt)
        for (const auto& [object_id, box] : objects) {
            const float iou = compute_iou_if_present(object_id, box, pred[file_id]);
            ++count;
            if (iou > 0.0f) total += iou;
            else if (log) *log << "No prediction for: " << object_id << "\n";
        }
    return count > 0 ? total / (float)count : 0.0f;
}

// metrics.cpp:12-26: mean over the class directories of the dataset of their IoU (directory order)
inline float compute_mean_intersection_over_union(const std::string& dataset, const std::string& output,
                                                  const std::string& gt_sub = "labels", std::ostream* log = nullptr) {
    namespace fs = std::filesystem;
    std::vector<float> per_class;
    for (const fs::directory_entry& c : fs::directory_iterator(dataset))
        if (c.is_directory())
            per_class.push_back(compute_intersection_over_union((c.path() / gt_sub).string(),
                                                                (fs::path(output) / c.path().filename()).string(), log));
    if (per_class.empty()) return 0.0f;
    return std::accumulate(per_class.begin(), per_class.end(), 0.0f) / (float)per_class.size();
}

// metrics.cpp:107-186: per class (object id up to its first '_'), the fraction of ground-truth
// objects whose same-id prediction in the same file has IoU >= 0.5
inline std::map<std::string, float> compute_detection_accuracy(const std::string& dataset, const std::string& output,
                                                               const std::string& gt_sub = "labels",
                                                               std::ostream* log = nullptr) {
    namespace fs = std::filesystem;
    std::map<std::string, int> total, tp;
    for (const fs::directory_entry& c : fs::directory_iterator(dataset)) {
        if (!c.is_directory()) continue;
        const BoxMap gt = read_boxes_coordinates((c.path() / gt_sub).string());
        BoxMap pred = read_boxes_coordinates((fs::path(output) / c.path().filename()).string());
        for (const auto& [file_id, objects] : gt)
            for (const auto& [object_id, box] : objects) {
                const std::string cls = object_id.substr(0, object_id.find('_'));
                ++total[cls];
                auto pf = pred.find(file_id);
                if (pf != pred.end() && pf->second.count(object_id)) {
                    if (compute_iou_if_present(object_id, box, pf->second) >= 0.5f) ++tp[cls];
                    else if (log) *log << "Object " << object_id << " in file " << file_id << " isn't a true positive\n";
                } else if (log) {
                    *log << "No prediction found for object " << object_id << " in file " << file_id << "\n";
                }
            }
    }
    std::map<std::string, float> acc;
    for (const auto& [cls, n] : total) acc[cls] = n > 0 ? (float)tp[cls] / (float)n : 0.0f;
    return acc;
}

}  // namespace mim
