/*
 * Types.h -- the value types of the C++ host layer (namespace ORB_SLAM2) over the gfx950 C ABI.
 *
 * The reference passes OpenCV types across the feature path (cv::Mat images and descriptor matrices,
 * cv::KeyPoint, cv::Point2f).  OpenCV is not part of this build, so the host layer uses these plain
 * equivalents with the same memory layout where the layout matters:
 *   KeyPoint  -- cv::KeyPoint's 28-byte layout {Point2f pt; float size, angle, response; int octave,
 *                class_id;} (== orbgpu_keypoint), so a std::vector<cv::KeyPoint> maps onto it in place;
 *   ImageU8   -- a CV_8UC1 cv::Mat: rows, cols, step (bytes per row), data; owning or a view;
 *   Descriptors -- the N x 32 CV_8U descriptor cv::Mat (row i = keypoint i);
 *   CameraMatrix / DistCoef -- the K (3x3 CV_32F) and mDistCoef (4 or 5 x 1 CV_32F) Mats the Frame
 *                constructors receive (src/Frame.cc:58-60, src/Tracking.cc:62-90).
 * INTEGRATION.md shows the few lines that convert cv:: objects into these at the ORB-SLAM2 boundary.
 */
#ifndef ORBSLAM2_GPU_TYPES_H
#define ORBSLAM2_GPU_TYPES_H

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../orbgpu.h"

namespace ORB_SLAM2
{

struct Point2f {
    float x = 0.f, y = 0.f;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};

struct KeyPoint {
    Point2f pt;
    float size = 0.f;
    float angle = -1.f;
    float response = 0.f;
    int octave = 0;
    int class_id = -1;
};
static_assert(sizeof(KeyPoint) == sizeof(orbgpu_keypoint), "KeyPoint must keep cv::KeyPoint's 28-byte layout");

/* Grey 8-bit image (CV_8UC1).  Owning images allocate rows*cols bytes (step == cols); views wrap caller
 * memory. */
class ImageU8
{
public:
    int rows = 0, cols = 0;
    size_t step = 0;
    uint8_t* data = nullptr;

    ImageU8() = default;
    ImageU8(int rows_, int cols_) { create(rows_, cols_); }
    static ImageU8 view(const uint8_t* p, int rows_, int cols_, size_t step_)
    {
        ImageU8 im;
        im.rows = rows_;
        im.cols = cols_;
        im.step = step_;
        im.data = const_cast<uint8_t*>(p);
        return im;
    }
    void create(int rows_, int cols_)
    {
        rows = rows_;
        cols = cols_;
        step = (size_t)cols_;
        buf_ = std::make_shared<std::vector<uint8_t>>((size_t)rows_ * (size_t)cols_);
        data = buf_->data();
    }
    bool empty() const { return rows == 0 || cols == 0 || data == nullptr; }
    uint8_t* ptr(int r) const { return data + (size_t)r * step; }

private:
    std::shared_ptr<std::vector<uint8_t>> buf_;
};

/* Depth map as the RGB-D Frame constructor receives it: CV_32F metres (is_u16 == false), or the raw
 * CV_16U sensor image that Tracking::GrabImageRGBD converts with convertTo(CV_32F, mDepthMapFactor)
 * (src/Tracking.cc:227-228); the GPU kernel fuses that conversion (factor = mDepthMapFactor). */
struct DepthImage {
    const void* data = nullptr;
    int rows = 0, cols = 0;
    size_t step = 0;  // bytes per row
    bool is_u16 = false;
    float factor = 1.0f;
};

/* N x 32 CV_8U descriptor matrix. */
class Descriptors
{
public:
    int rows = 0;
    std::vector<uint8_t> buf;
    static constexpr int cols = 32;

    bool empty() const { return rows == 0; }
    void create(int n)
    {
        rows = n;
        buf.resize((size_t)n * 32);
    }
    void release()
    {
        rows = 0;
        buf.clear();
    }
    const uint8_t* row(int i) const { return buf.data() + (size_t)i * 32; }
    uint8_t* row(int i) { return buf.data() + (size_t)i * 32; }
    const uint8_t* data() const { return buf.data(); }
    uint8_t* data() { return buf.data(); }
};

/* K = [fx 0 cx; 0 fy cy; 0 0 1] as float (K.at<float>(0,0) ... in the reference). */
struct CameraMatrix {
    float fx = 0.f, fy = 0.f, cx = 0.f, cy = 0.f;
};

/* mDistCoef: k1, k2, p1, p2[, k3] (0, 4 or 5 entries). */
using DistCoef = std::vector<float>;

/* 4x4 row-major float pose Tcw (cv::Mat 4x4 CV_32F in the reference). */
struct Pose {
    float T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    bool empty = true;
};

/* Thrown where the reference would fail an assert or where the HIP runtime reports an error; the
 * reference itself has no error channel on this path. */
class GpuError : public std::runtime_error
{
public:
    explicit GpuError(const std::string& what) : std::runtime_error(what) {}
};

}  // namespace ORB_SLAM2

#endif
