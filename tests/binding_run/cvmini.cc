// tests/binding_run/cvmini.cc -- the minimal cv::Mat / InputArray / OutputArray behaviour the drop-in
// integration/ORBextractor.cc relies on, defined over integration/cvshim's declarations so that the binding can be
// linked and executed in a test (tests/test_gpu_binding_run.py).  Test infrastructure: not OpenCV, not shipped.
// Only 8-bit single-channel matrices occur (CV_8U images, the N x 32 descriptor matrix, the pyramid levels).
#include <cstring>
#include <stdexcept>

#include "opencv2/core/core.hpp"

namespace cv {

Mat::Mat() : rows(0), cols(0), step(0), data(nullptr) {}

Mat::Mat(int r, int c, int t) : Mat() { create(r, c, t); }

Mat::Mat(int r, int c, int t, void* d, size_t s)
    : rows(r), cols(c), step(s ? s : (size_t)c), data(static_cast<unsigned char*>(d)), type_(t)
{
}

bool Mat::empty() const { return data == nullptr || rows == 0 || cols == 0; }
int Mat::type() const { return type_; }
bool Mat::isContinuous() const { return step == (size_t)cols || rows <= 1; }

void Mat::create(int r, int c, int t)
{
    if (t != CV_8U) throw std::invalid_argument("cvmini: 8-bit single-channel matrices only");
    if (buf_ && r == rows && c == cols && t == type_) return;  // cv::Mat::create keeps matching storage
    buf_.reset(new unsigned char[(size_t)r * c + 1](), std::default_delete<unsigned char[]>());
    rows = r;
    cols = c;
    step = (size_t)c;
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

void Mat::copyTo(OutputArray o) const
{
    o.create(rows, cols, type_);
    Mat& d = o.getMatRef();
    for (int r = 0; r < rows; r++) std::memcpy(d.data + (size_t)r * d.step, data + (size_t)r * step, (size_t)cols);
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
