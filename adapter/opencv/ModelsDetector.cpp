// Drop-in replacement of the reference's src/ModelsDetector.cpp with SIFT on the MI355X (built with
// MIM_GPU_SIFT; same function and signature, /root/reference/include/ModelsDetector.hpp:13-14):
//
//   void processAllModelsImages(const std::string& basePath, std::vector<ObjectModel>& models,
//                               cv::Ptr<cv::Feature2D>& detector);
//
// Behaviour kept from the reference (ModelsDetector.cpp:14-86): one ObjectModel per sub-folder of
// basePath in directory order; its views are the "<base>_color*" files of <folder>/models/, each
// paired with "<base>_mask*"; views are visited in the iteration order of the same
// std::unordered_map<std::string, std::string> the reference fills (so the same view order on the
// same standard library); gray image and mask read with IMREAD_GRAYSCALE, preprocessImage applied;
// the same messages for a missing base path, an unreadable image or mask, a missing mask.
// What changes: detectAndCompute (:75) runs on the device (mim_sift_detect_compute with the view's
// mask), SIFT::create()'s defaults, which is the detector main.cpp:17 passes; `detector` is not called.
#include "ModelsDetector.hpp"

#include <filesystem>
#include <iostream>
#include <unordered_map>

#include "mim_device.hpp"
#include "preprocessing.hpp"

namespace {

// mim_keypoint -> cv::KeyPoint (pt, size, angle, response, octave; class_id -1 as SIFT leaves it)
std::vector<cv::KeyPoint> to_cv(const std::vector<mim_keypoint>& k) {
    std::vector<cv::KeyPoint> out;
    out.reserve(k.size());
    for (const mim_keypoint& p : k) out.emplace_back(p.x, p.y, p.size, p.angle, p.response, p.octave);
    return out;
}

ObjectModel describe_folder(const std::filesystem::path& folder) {
    ObjectModel model;
    model.name = folder.filename().string();
    std::unordered_map<std::string, std::string> color, mask;  // base name -> path
    for (const auto& f : std::filesystem::directory_iterator(folder.string() + "/models/")) {
        const std::string file = f.path().filename().string();
        if (const size_t c = file.find("_color"); c != std::string::npos)
            color[file.substr(0, c)] = f.path().string();
        else if (const size_t m = file.find("_mask"); m != std::string::npos)
            mask[file.substr(0, m)] = f.path().string();
    }
    for (const auto& [base, path] : color) {
        const cv::Mat img = cv::imread(path, cv::IMREAD_GRAYSCALE);
        if (img.empty()) {
            std::cout << "Error loading image: " << path << std::endl;
            continue;
        }
        cv::Mat m;
        if (const auto it = mask.find(base); it == mask.end()) {
            std::cout << "Mask not found for: " << base << std::endl;
        } else if ((m = cv::imread(it->second, cv::IMREAD_GRAYSCALE)).empty()) {
            std::cout << "Error loading mask: " << it->second << std::endl;
        }
        const cv::Mat gray = preprocessImage(img);
        CV_Assert(gray.type() == CV_8UC1 && (m.empty() || (m.type() == CV_8UC1 && m.size() == gray.size())));
        std::vector<mim_keypoint> kps;
        std::vector<float> desc;
        mim_device().sift(gray.data, gray.rows, gray.cols, (int64_t)gray.step[0], m.empty() ? nullptr : m.data,
                          m.empty() ? 0 : (int64_t)m.step[0], kps, desc);
        cv::Mat d((int)kps.size(), 128, CV_32F);
        if (!kps.empty()) std::copy(desc.begin(), desc.end(), d.ptr<float>());
        model.images.push_back(img);
        model.keypoints.push_back(to_cv(kps));
        model.descriptors.push_back(kps.empty() ? cv::Mat() : d);
    }
    return model;
}

}  // namespace

void processAllModelsImages(const std::string& basePath, std::vector<ObjectModel>& models,
                            cv::Ptr<cv::Feature2D>& detector) {
    (void)detector;
    if (!std::filesystem::exists(basePath)) {
        std::cout << "Error: basePath does not exist: " << basePath << std::endl;
        return;
    }
    for (const auto& entry : std::filesystem::directory_iterator(basePath))
        if (std::filesystem::is_directory(entry)) models.push_back(describe_folder(entry.path()));
}
