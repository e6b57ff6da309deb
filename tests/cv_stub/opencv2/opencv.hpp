// COMPILE-CHECK STUB, test infrastructure only (tests/test_adapter_compile.py): declarations of the
// few OpenCV 4 names the reference's headers and adapter/opencv/*.cpp use, so that `g++ -fsyntax-only`
// can type-check the adapter in this image, which has no OpenCV.  Nothing here is defined, linked,
// shipped or used to replace OpenCV; the adapter builds against the real OpenCV (CMake MIM_WITH_OPENCV).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#define CV_8U 0
#define CV_32F 5
#define CV_8UC1 CV_8U
#define CV_Assert(expr) ((void)(expr))

namespace cv {
typedef unsigned char uchar;
struct Point2f {
    float x, y;
};
struct Size {
    int width = 0, height = 0;
    Size() = default;
    Size(int w, int h) : width(w), height(h) {}
    bool operator==(const Size& o) const { return width == o.width && height == o.height; }
};
struct Rect {
    int x, y, width, height;
    Rect(int x_, int y_, int w, int h) : x(x_), y(y_), width(w), height(h) {}
};
struct KeyPoint {
    KeyPoint(float x, float y, float size, float angle = -1, float response = 0, int octave = 0, int class_id = -1);
    Point2f pt;
    float size, angle, response;
    int octave, class_id;
};
struct MatStep {
    size_t operator[](int i) const;
    operator size_t() const;
};
class Mat {
   public:
    Mat();
    Mat(int rows, int cols, int type);
    bool empty() const;
    int type() const;
    bool isContinuous() const;
    Mat clone() const;
    size_t total() const;
    Size size() const;
    template <class T> T* ptr(int row = 0);
    template <class T> const T* ptr(int row = 0) const;
    int rows, cols;
    uchar* data;
    MatStep step;
};
class _InputArray {
   public:
    _InputArray(const Mat&);
};
typedef const _InputArray& InputArray;
class _OutputArray {
   public:
    _OutputArray(Mat&);
    _OutputArray(std::vector<KeyPoint>&);
};
typedef const _OutputArray& OutputArray;
InputArray noArray();
template <class T> class Ptr {
   public:
    T* operator->() const;
};
class Feature2D {
   public:
    virtual ~Feature2D();
    virtual void detectAndCompute(InputArray image, InputArray mask, std::vector<KeyPoint>& keypoints,
                                  OutputArray descriptors, bool useProvidedKeypoints = false);
};
enum { IMREAD_GRAYSCALE = 0, IMREAD_COLOR = 1 };
Mat imread(const std::string& filename, int flags = IMREAD_COLOR);
void resize(InputArray src, OutputArray dst, Size dsize, double fx = 0, double fy = 0, int interpolation = 1);
}  // namespace cv
