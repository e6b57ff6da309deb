// mim_types.hpp — the two plain geometry types the host layer shares (OpenCV-free stand-ins for
// cv::Point2f and cv::Rect: same members, same arithmetic types).
#pragma once

namespace mim {

struct Point2f {  // cv::Point2f (KeyPoint::pt, the scene points of TestsDetector.cpp:39)
    float x, y;
};

struct Rect {  // cv::Rect: top-left corner + size, integers
    int x, y, width, height;
};

}  // namespace mim
