// Test shim for the drop-in binding (not OpenCV, not part of the product): declarations of the cv:: names the
// integration/ sources and the reference's include/ORBextractor.h use.  tests/test_integration_compile.py compiles
// the binding against them (g++ -fsyntax-only); tests/binding_run/cvmini.cc defines the subset the replacement
// ORBextractor.cc calls, so tests/binding_run/run_binding executes the binding itself on the GPU
// (tests/test_gpu_binding_run.py).  The private members below are that minimal implementation's storage.
#pragma once
#include <cstddef>
#include <memory>
#include <vector>

#define CV_8U 0
#define CV_8UC1 0
#define CV_32F 5

namespace cv {
template <typename T>
struct Point_ {
    T x, y;
};
typedef Point_<int> Point2i;
typedef Point2i Point;
typedef Point_<float> Point2f;

struct KeyPoint {
    Point2f pt;
    float size, angle, response;
    int octave, class_id;
};

struct Range {
    int start, end;
};

class _OutputArray;
typedef const _OutputArray& OutputArray;

class Mat {
public:
    Mat();
    Mat(int rows, int cols, int type);
    Mat(int rows, int cols, int type, void* data, size_t step = 0);
    int rows, cols;
    size_t step;
    unsigned char* data;
    bool empty() const;
    int type() const;
    bool isContinuous() const;
    void create(int rows, int cols, int type);
    void release();
    Mat clone() const;
    void copyTo(OutputArray m) const;
    Mat rowRange(int a, int b) const;
    Mat colRange(int a, int b) const;
    Mat col(int c) const;
    Mat t() const;
    template <typename T>
    T& at(int i, int j = 0);
    template <typename T>
    const T& at(int i, int j = 0) const;
    template <typename T>
    T* ptr(int i = 0);
    template <typename T>
    const T* ptr(int i = 0) const;

private:
    int type_ = 0;
    std::shared_ptr<unsigned char> buf_;  // owned storage (shared by copies, as OpenCV's reference count)
};

class _InputArray {
public:
    _InputArray();
    _InputArray(const Mat& m);
    bool empty() const;
    Mat getMat() const;

protected:
    const Mat* m_ = nullptr;
};
class _OutputArray : public _InputArray {
public:
    _OutputArray();
    _OutputArray(Mat& m);
    void release() const;
    void create(int rows, int cols, int type) const;
    Mat& getMatRef() const;

private:
    Mat* out_ = nullptr;
};
typedef const _InputArray& InputArray;
// matrix expressions (OpenCV returns MatExpr, which converts to Mat) and cv::norm (default NORM_L2)
Mat operator-(const Mat& a);
Mat operator-(const Mat& a, const Mat& b);
Mat operator*(const Mat& a, const Mat& b);
double norm(InputArray src1, int normType = 4);
}  // namespace cv
