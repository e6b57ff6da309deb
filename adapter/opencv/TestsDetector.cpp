// Drop-in replacement of the reference's src/TestsDetector.cpp: same function, same signature
// (/root/reference/include/TestsDetector.hpp:13-17), the matcher + RANSAC hot path on the MI355X.
//
//   std::vector<std::pair<cv::Rect, std::string>> detectObjects(const cv::Mat& scene,
//       const std::vector<ObjectModel>& models, cv::Ptr<cv::Feature2D>& detector);
//
// What changes against the reference (TestsDetector.cpp:15-279):
//   * the scene is converted (preprocessImage), resized and SIFT-described ONCE per scale (:99-107),
//     not once per scale per model: SIFT is deterministic, so every model sees
//     the keypoints/descriptors the reference computes for it;
//   * with MIM_GPU_SIFT (CMake -DMIM_GPU_SIFT=ON) the five resizes and SIFT runs of :102,106 happen on
//     the device in one call whose descriptors stay there as the batch's scene sets
//     (mim::Detector::detect_scene_gray over mim_sift_scales_sets: the scene uploaded once), and
//     adapter/opencv/ModelsDetector.cpp describes the model views on the device too
//     (ModelsDetector.cpp:75).  libmim's SIFT is SIFT::create() with its defaults (main.cpp:17), which is
//     the detector the reference always passes; `detector` is then not called;
//   * every (model, view, scale) problem of the scene — knnMatch k=2 (:60), ratio test (:66-72),
//     gates (:74, :79, :81, :84), findHomography RANSAC (:78), inlier gather and 1/scale (:87-94) —
//     runs as ONE device batch through libmim (mim::Detector::detect_scene, include/mim.hpp);
//   * clustering, margins, merging and the area gate (:111-248) run through include/mim_detect.hpp,
//     which keeps the reference's std::unordered_set visiting order (identical clusters and boxes);
//   * the visualisation of :250-273 is not reproduced: it draws into a local clone of the scene that
//     the reference never returns or writes.
// The "Rejected box ..." messages (:242-244) go to std::cout as in the reference.
//
// Built by the CMake target `mim_opencv` (CMakeLists.txt, -DMIM_WITH_OPENCV=ON) together with the
// reference's other sources; see INTEGRATION.md §2.  OpenCV is absent from this image, so this file
// is compiled only where OpenCV is installed; the code it delegates to (mim.hpp, mim_detect.hpp) is
// built and tested here (tests/cpp/test_mim_hpp.cpp, tests/cpp/test_detect.cpp).
#include "TestsDetector.hpp"

#include <iostream>
#include <unordered_map>

#include "mim_detect.hpp"
#include "mim_device.hpp"
#include "preprocessing.hpp"

namespace {

// ObjectModel (objectModel.hpp:11-16) -> mim::ModelViews: CV_32F descriptor rows + KeyPoint::pt
mim::ModelViews to_views(const ObjectModel& m) {
    mim::ModelViews mv{m.name, {}};
    mv.views.reserve(m.descriptors.size());
    for (size_t v = 0; v < m.descriptors.size(); ++v) {
        mim::View view;
        const cv::Mat& d = m.descriptors[v];
        if (!d.empty()) {
            CV_Assert(d.type() == CV_32F && d.cols == 128);
            const cv::Mat dc = d.isContinuous() ? d : d.clone();
            view.descriptors.assign(dc.ptr<float>(), dc.ptr<float>() + dc.total());
        }
        view.keypoints.reserve(m.keypoints[v].size());
        for (const cv::KeyPoint& k : m.keypoints[v]) view.keypoints.push_back({k.pt.x, k.pt.y});
        mv.views.push_back(std::move(view));
    }
    return mv;
}

// the converted models, kept across scenes (the models are loaded once, main.cpp:22).  Keyed by the
// ObjectModel's address AND the data pointers and sizes of its descriptor matrices and keypoint
// vectors, so a different model that happens to reuse a freed address, or a model whose keypoints were
// replaced while its descriptor Mats kept their buffers, is converted anew.
const mim::ModelViews& views_of(const ObjectModel& m) {
    struct Entry {
        std::vector<std::pair<const void*, size_t>> key;
        mim::ModelViews views;
    };
    static std::unordered_map<const ObjectModel*, Entry> cache;
    std::vector<std::pair<const void*, size_t>> key;
    key.reserve(m.descriptors.size() + m.keypoints.size());
    for (const cv::Mat& d : m.descriptors) key.emplace_back(static_cast<const void*>(d.data), d.total());
    for (const std::vector<cv::KeyPoint>& k : m.keypoints) key.emplace_back(static_cast<const void*>(k.data()), k.size());
    auto it = cache.find(&m);
    if (it == cache.end() || it->second.key != key) it = cache.insert_or_assign(&m, Entry{key, to_views(m)}).first;
    return it->second.views;
}

}  // namespace

std::vector<std::pair<cv::Rect, std::string>> detectObjects(const cv::Mat& scene, const std::vector<ObjectModel>& models,
                                                            cv::Ptr<cv::Feature2D>& detector) {
    const mim::BoxParams box_params;  // TestsDetector.cpp:26-30
    const cv::Mat preprocessed = preprocessImage(scene);

    // :38-109 for every model at once: one device batch of all (model, scale, view) problems, the
    // scene described once per scale for all models (:99-107)
    const std::vector<float> scales = {0.7f, 0.85f, 1.0f, 1.15f, 1.3f};
    std::vector<const mim::ModelViews*> mv;
    for (const ObjectModel& m : models) mv.push_back(&views_of(m));
    std::vector<std::vector<mim::Point2f>> all_pts;  // allUnfilteredScenePts per model (:39)
#ifdef MIM_GPU_SIFT
    (void)detector;  // SIFT::create() defaults, on the device
    CV_Assert(preprocessed.type() == CV_8UC1);
    mim_device().detect_scene_gray(mv, preprocessed.data, preprocessed.rows, preprocessed.cols,
                                   (int64_t)preprocessed.step[0], scales, all_pts);
#else
    std::vector<std::vector<mim::Point2f>> scene_kp(scales.size());
    std::vector<std::vector<float>> scene_desc(scales.size());
    for (size_t s = 0; s < scales.size(); ++s) {
        cv::Mat scaled;
        cv::resize(preprocessed, scaled, cv::Size(), scales[s], scales[s]);
        std::vector<cv::KeyPoint> kp;
        cv::Mat desc;
        detector->detectAndCompute(scaled, cv::noArray(), kp, desc);
        for (const cv::KeyPoint& k : kp) scene_kp[s].push_back({k.pt.x, k.pt.y});
        if (!desc.empty()) {
            CV_Assert(desc.type() == CV_32F && desc.cols == 128);
            const cv::Mat dc = desc.isContinuous() ? desc : desc.clone();
            scene_desc[s].assign(dc.ptr<float>(), dc.ptr<float>() + dc.total());
        }
    }
    std::vector<mim::Detector::ScaledScene> ss;
    for (size_t s = 0; s < scales.size(); ++s) ss.push_back({&scene_kp[s], &scene_desc[s], scales[s]});
    mim_device().detect_scene(mv, ss, all_pts);
#endif

    // :111-248 per model, in model order
    mim::Detections dets;
    for (size_t m = 0; m < models.size(); ++m) mim::boxes_for_model(all_pts[m], models[m].name, dets, box_params, &std::cout);
    std::vector<std::pair<cv::Rect, std::string>> out;
    out.reserve(dets.size());
    for (const auto& [b, name] : dets) out.emplace_back(cv::Rect(b.x, b.y, b.width, b.height), name);
    return out;
}
