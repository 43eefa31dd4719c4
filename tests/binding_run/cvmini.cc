// tests/binding_run/cvmini.cc -- the minimal cv::Mat / InputArray / OutputArray behaviour the drop-in
// integration/ sources rely on, defined over integration/cvshim's declarations so that the bindings can be linked
// and executed in a test (tests/test_gpu_binding_run.py).  Test infrastructure: not OpenCV, not shipped.
// Single-channel matrices only: CV_8U (images, the N x 32 descriptor matrix, the pyramid levels) and CV_32F (the
// 4x4 pose mTcw, 3x1 positions).  The float expressions follow OpenCV's baseline build, without FMA contraction
// (built with -ffp-contract=off): A * B sums the products in k order in float (((a0 b0 + a1 b1) + a2 b2), as
// OpenCV's small-matrix gemm), cv::norm accumulates squares in double.
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "opencv2/core/core.hpp"

namespace cv {

Mat::Mat() : rows(0), cols(0), step(0), data(nullptr) {}

Mat::Mat(int r, int c, int t) : Mat() { create(r, c, t); }

static size_t elem_size(int t)
{
    if (t == CV_8U) return 1;
    if (t == CV_32F) return 4;
    throw std::invalid_argument("cvmini: CV_8U or CV_32F single-channel matrices only");
}

Mat::Mat(int r, int c, int t, void* d, size_t s)
    : rows(r), cols(c), step(s ? s : (size_t)c * elem_size(t)), data(static_cast<unsigned char*>(d)), type_(t)
{
}

bool Mat::empty() const { return data == nullptr || rows == 0 || cols == 0; }
int Mat::type() const { return type_; }
bool Mat::isContinuous() const { return step == (size_t)cols || rows <= 1; }

void Mat::create(int r, int c, int t)
{
    const size_t es = elem_size(t);
    // cv::Mat::create keeps matching storage, its own or a header over the caller's data
    if (data && r == rows && c == cols && t == type_) return;
    buf_.reset(new unsigned char[(size_t)r * c * es + 1](), std::default_delete<unsigned char[]>());
    rows = r;
    cols = c;
    step = (size_t)c * es;
    type_ = t;
    data = buf_.get();
}

void Mat::release()
{
    buf_.reset();
    rows = cols = 0;
    step = 0;
    data = nullptr;
}

Mat Mat::rowRange(int a, int b) const
{
    Mat m(*this);  // shares the storage
    m.rows = b - a;
    m.data = data + (size_t)a * step;
    return m;
}

Mat Mat::colRange(int a, int b) const
{
    Mat m(*this);
    m.cols = b - a;
    m.data = data + (size_t)a * elem_size(type_);
    return m;
}

Mat Mat::col(int c) const { return colRange(c, c + 1); }

Mat Mat::clone() const
{
    Mat m;
    Mat& r = m;
    copyTo(r);
    return m;
}

void Mat::copyTo(OutputArray o) const
{
    o.create(rows, cols, type_);
    Mat& d = o.getMatRef();
    const size_t w = (size_t)cols * elem_size(type_);
    for (int r = 0; r < rows; r++) std::memcpy(d.data + (size_t)r * d.step, data + (size_t)r * step, w);
}

template <typename T>
T& Mat::at(int i, int j)
{
    return reinterpret_cast<T*>(data + (size_t)i * step)[j];
}
template <typename T>
const T& Mat::at(int i, int j) const
{
    return reinterpret_cast<const T*>(data + (size_t)i * step)[j];
}
template <typename T>
T* Mat::ptr(int i)
{
    return reinterpret_cast<T*>(data + (size_t)i * step);
}
template <typename T>
const T* Mat::ptr(int i) const
{
    return reinterpret_cast<const T*>(data + (size_t)i * step);
}
template float& Mat::at<float>(int, int);
template const float& Mat::at<float>(int, int) const;
template unsigned char& Mat::at<unsigned char>(int, int);
template const unsigned char& Mat::at<unsigned char>(int, int) const;
template float* Mat::ptr<float>(int);
template const float* Mat::ptr<float>(int) const;
template unsigned char* Mat::ptr<unsigned char>(int);
template const unsigned char* Mat::ptr<unsigned char>(int) const;

static void need_f32(const Mat& a)
{
    if (a.type() != CV_32F) throw std::invalid_argument("cvmini: matrix expressions on CV_32F only");
}

Mat Mat::t() const
{
    need_f32(*this);
    Mat m(cols, rows, CV_32F);
    for (int i = 0; i < rows; i++)
        for (int j = 0; j < cols; j++) m.at<float>(j, i) = at<float>(i, j);
    return m;
}

Mat operator-(const Mat& a)
{
    need_f32(a);
    Mat m(a.rows, a.cols, CV_32F);
    for (int i = 0; i < a.rows; i++)
        for (int j = 0; j < a.cols; j++) m.at<float>(i, j) = -a.at<float>(i, j);
    return m;
}

Mat operator-(const Mat& a, const Mat& b)
{
    need_f32(a);
    need_f32(b);
    if (a.rows != b.rows || a.cols != b.cols) throw std::invalid_argument("cvmini: size mismatch");
    Mat m(a.rows, a.cols, CV_32F);
    for (int i = 0; i < a.rows; i++)
        for (int j = 0; j < a.cols; j++) m.at<float>(i, j) = a.at<float>(i, j) - b.at<float>(i, j);
    return m;
}

Mat operator*(const Mat& a, const Mat& b)
{
    need_f32(a);
    need_f32(b);
    if (a.cols != b.rows) throw std::invalid_argument("cvmini: size mismatch");
    Mat m(a.rows, b.cols, CV_32F);
    for (int i = 0; i < a.rows; i++)
        for (int j = 0; j < b.cols; j++) {
            float s = a.at<float>(i, 0) * b.at<float>(0, j);
            for (int k = 1; k < a.cols; k++) s = s + a.at<float>(i, k) * b.at<float>(k, j);
            m.at<float>(i, j) = s;
        }
    return m;
}

double norm(InputArray src, int normType)
{
    if (normType != 4) throw std::invalid_argument("cvmini: NORM_L2 only");
    const Mat a = src.getMat();
    need_f32(a);
    double ss = 0.0;
    for (int i = 0; i < a.rows; i++)
        for (int j = 0; j < a.cols; j++) ss += (double)a.at<float>(i, j) * (double)a.at<float>(i, j);
    return std::sqrt(ss);
}

_InputArray::_InputArray() {}
_InputArray::_InputArray(const Mat& m) : m_(&m) {}
bool _InputArray::empty() const { return !m_ || m_->empty(); }
Mat _InputArray::getMat() const { return m_ ? *m_ : Mat(); }

_OutputArray::_OutputArray() {}
_OutputArray::_OutputArray(Mat& m) : _InputArray(m), out_(&m) {}
void _OutputArray::release() const
{
    if (out_) out_->release();
}
void _OutputArray::create(int r, int c, int t) const
{
    if (!out_) throw std::invalid_argument("cvmini: no output matrix");
    out_->create(r, c, t);
}
Mat& _OutputArray::getMatRef() const
{
    if (!out_) throw std::invalid_argument("cvmini: no output matrix");
    return *out_;
}

}  // namespace cv
