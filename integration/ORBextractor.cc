// integration/ORBextractor.cc -- drop-in replacement for the reference's src/ORBextractor.cc.
//
// Compiles against the reference's UNCHANGED include/ORBextractor.h (tests/test_integration_compile.py checks that
// with the declarations of integration/cvshim) and links against liborbgpu.so (include/orbgpu.h).  The class
// keeps its constructor, operator(), getters and the public mvImagePyramid (include/ORBextractor.h:45-111); the
// private helpers (ComputePyramid, ComputeKeyPointsOctTree, DistributeOctTree, DivideNode) stay declared and
// are no longer defined or called -- the whole of operator() runs on the GPU (src/ORBextractor.cc:1043-1105).
#include <cassert>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <unordered_map>

#include "ORBextractor.h"
#include "orbgpu.h"
#include "orbgpu_binding.h"

namespace ORB_SLAM2 {

static_assert(sizeof(cv::KeyPoint) == sizeof(orbgpu_keypoint), "cv::KeyPoint layout");

// Linked from integration/Frame_stereo.cc when that replacement is part of the build: ComputeStereoMatches then reads
// both pyramids in device memory and nothing else in ORB-SLAM2 reads mvImagePyramid (src/Frame.cc:473,563,575,580).
extern "C" __attribute__((weak)) const int orbgpu_binding_device_stereo;

namespace {
struct Entry {
    orbgpu_ctx* ctx;
    bool host_pyramid;  // refresh mvImagePyramid after each call
};
std::mutex g_mu;
std::unordered_map<const ORBextractor*, Entry>& contexts()
{
    static std::unordered_map<const ORBextractor*, Entry> m;
    return m;
}

int env_int(const char* name, int dflt)
{
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

// Default for new extractors: download the pyramid only if something may read it -- i.e. unless the device stereo
// matcher is linked; ORBGPU_HOST_PYRAMID=0/1 overrides (about 3 MB per 1080p frame over PCIe when on)
bool default_host_pyramid()
{
    return env_int("ORBGPU_HOST_PYRAMID", &orbgpu_binding_device_stereo == nullptr ? 1 : 0) != 0;
}
}  // namespace

orbgpu_ctx* orbgpu_context_of(const ORBextractor* ex)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = contexts().find(ex);
    return it == contexts().end() ? nullptr : it->second.ctx;
}

void orbgpu_release_extractor(const ORBextractor* ex)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = contexts().find(ex);
    if (it == contexts().end()) return;
    orbgpu_destroy(it->second.ctx);
    contexts().erase(it);
}

void orbgpu_set_host_pyramid(const ORBextractor* ex, bool on)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = contexts().find(ex);
    if (it != contexts().end()) it->second.host_pyramid = on;
}

// src/ORBextractor.cc:410-470: the scale tables and per-level budgets come from the context (same arithmetic)
ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST)
{
    // device: ORBGPU_DEVICE (default 0), e.g. one SLAM process per GPU
    orbgpu_ctx* ctx = orbgpu_create(env_int("ORBGPU_DEVICE", 0), nfeatures, _scaleFactor, nlevels, iniThFAST,
                                    minThFAST);
    if (!ctx) throw std::runtime_error("orbgpu_create failed (no gfx950 device, or invalid parameters)");
    {
        // the reference header's inline ~ORBextractor() cannot release the context: an extractor constructed at
        // the address of a deleted one takes over the slot, and the old context is destroyed here
        // (orbgpu_release_extractor releases one explicitly)
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = contexts().find(this);
        if (it != contexts().end()) orbgpu_destroy(it->second.ctx);
        contexts()[this] = Entry{ctx, default_host_pyramid()};
    }
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    orbgpu_get_scale_factors(ctx, mvScaleFactor.data());
    orbgpu_get_inverse_scale_factors(ctx, mvInvScaleFactor.data());
    orbgpu_get_scale_sigma_squares(ctx, mvLevelSigma2.data());
    orbgpu_get_inverse_scale_sigma_squares(ctx, mvInvLevelSigma2.data());
    orbgpu_get_features_per_level(ctx, mnFeaturesPerLevel.data());
    mvImagePyramid.resize(nlevels);
}

// src/ORBextractor.cc:1043-1105 (mask ignored, as in the reference)
void ORBextractor::operator()(cv::InputArray _image, cv::InputArray _mask, std::vector<cv::KeyPoint>& _keypoints,
                              cv::OutputArray _descriptors)
{
    (void)_mask;
    if (_image.empty()) return;  // :1046-1047, outputs untouched
    cv::Mat image = _image.getMat();
    assert(image.type() == CV_8UC1);
    orbgpu_ctx* ctx = orbgpu_context_of(this);
    int cap = orbgpu_max_keypoints(ctx), n = 0;
    _keypoints.resize(cap);
    cv::Mat desc(cap, 32, CV_8U);
    int rc = orbgpu_extract(ctx, image.data, image.cols, image.rows, image.step,
                            reinterpret_cast<orbgpu_keypoint*>(_keypoints.data()), desc.data, cap, &n);
    if (rc == ORBGPU_ERR_CAPACITY) {
        cap = n;
        _keypoints.resize(cap);
        desc.create(cap, 32, CV_8U);
        rc = orbgpu_extract(ctx, image.data, image.cols, image.rows, image.step,
                            reinterpret_cast<orbgpu_keypoint*>(_keypoints.data()), desc.data, cap, &n);
    }
    if (rc != ORBGPU_OK) throw std::runtime_error(orbgpu_last_error(ctx));
    _keypoints.resize(n);
    if (n == 0) {
        _descriptors.release();  // :1064-1065
    } else {
        desc.rowRange(0, n).copyTo(_descriptors);
    }
    // the public mvImagePyramid (include/ORBextractor.h:85), read only by Frame::ComputeStereoMatches
    // (src/Frame.cc:473,563,575,580): downloaded when that reader may run on the CPU (default_host_pyramid)
    bool host_pyramid;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        host_pyramid = contexts()[this].host_pyramid;
    }
    if (!host_pyramid) return;
    for (int l = 0; l < nlevels; ++l) {
        int w = 0, h = 0;
        orbgpu_get_level(ctx, l, nullptr, 0, &w, &h);
        mvImagePyramid[l].create(h, w, CV_8U);
        orbgpu_get_level(ctx, l, mvImagePyramid[l].data, mvImagePyramid[l].step, &w, &h);
    }
}

}  // namespace ORB_SLAM2
