// ORB_SLAM2::ORBextractor over the gfx950 C ABI -- include/orbslam2_gpu/ORBextractor.h.
// Reference: include/ORBextractor.h:45-111, src/ORBextractor.cc:410-470 (constructor), :1043-1105 (operator()).
#include "orbslam2_gpu/ORBextractor.h"

#include <string>

namespace ORB_SLAM2
{

void orbgpu_throw_if(orbgpu_ctx* ctx, int rc, const char* what)
{
    if (rc == ORBGPU_OK) return;
    std::string msg = std::string(what) + " failed (status " + std::to_string(rc) + ")";
    if (ctx) msg += ": " + std::string(orbgpu_last_error(ctx));
    throw GpuError(msg);
}

ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST,
                           int device)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels), iniThFAST(_iniThFAST),
      minThFAST(_minThFAST)
{
    mCtx = orbgpu_create(device, nfeatures, _scaleFactor, nlevels, iniThFAST, minThFAST);
    if (!mCtx)
        throw GpuError("orbgpu_create failed: no gfx950 HIP device, or invalid extractor parameters "
                       "(the feature path has no CPU fallback)");
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    orbgpu_throw_if(mCtx, orbgpu_get_scale_factors(mCtx, mvScaleFactor.data()), "orbgpu_get_scale_factors");
    orbgpu_throw_if(mCtx, orbgpu_get_inverse_scale_factors(mCtx, mvInvScaleFactor.data()),
                    "orbgpu_get_inverse_scale_factors");
    orbgpu_throw_if(mCtx, orbgpu_get_scale_sigma_squares(mCtx, mvLevelSigma2.data()), "orbgpu_get_scale_sigma_squares");
    orbgpu_throw_if(mCtx, orbgpu_get_inverse_scale_sigma_squares(mCtx, mvInvLevelSigma2.data()),
                    "orbgpu_get_inverse_scale_sigma_squares");
    orbgpu_throw_if(mCtx, orbgpu_get_features_per_level(mCtx, mnFeaturesPerLevel.data()),
                    "orbgpu_get_features_per_level");
    mvImagePyramid.resize(nlevels);
}

ORBextractor::~ORBextractor()
{
    if (mCtx) orbgpu_destroy(mCtx);
}

void ORBextractor::operator()(const ImageU8& image, const ImageU8& /*mask: ignored, as in the reference*/,
                              std::vector<KeyPoint>& keypoints, Descriptors& descriptors)
{
    if (image.empty()) return;  // src/ORBextractor.cc:1046-1047: outputs untouched
    int cap = orbgpu_max_keypoints(mCtx), n = 0;
    std::vector<KeyPoint> kps((size_t)cap);
    Descriptors desc;
    desc.create(cap);
    int rc = orbgpu_extract(mCtx, image.data, image.cols, image.rows, image.step,
                            reinterpret_cast<orbgpu_keypoint*>(kps.data()), desc.data(), cap, &n);
    if (rc == ORBGPU_ERR_CAPACITY) {  // more keypoints than the pre-first-frame estimate
        cap = n;
        kps.resize((size_t)cap);
        desc.create(cap);
        rc = orbgpu_extract(mCtx, image.data, image.cols, image.rows, image.step,
                            reinterpret_cast<orbgpu_keypoint*>(kps.data()), desc.data(), cap, &n);
    }
    orbgpu_throw_if(mCtx, rc, "orbgpu_extract");
    kps.resize((size_t)n);
    keypoints.swap(kps);  // src/ORBextractor.cc:1072-1073 clears and refills the caller's vector
    if (n == 0) {
        descriptors.release();  // src/ORBextractor.cc:1064-1065
    } else {
        desc.rows = n;
        desc.buf.resize((size_t)n * 32);
        descriptors = std::move(desc);
    }
    if (mbDownloadPyramid) {
        for (int l = 0; l < nlevels; ++l) {
            int w = 0, h = 0;
            orbgpu_throw_if(mCtx, orbgpu_get_level(mCtx, l, nullptr, 0, &w, &h), "orbgpu_get_level");
            if (mvImagePyramid[l].rows != h || mvImagePyramid[l].cols != w) mvImagePyramid[l].create(h, w);
            orbgpu_throw_if(mCtx, orbgpu_get_level(mCtx, l, mvImagePyramid[l].data, mvImagePyramid[l].step, &w, &h),
                            "orbgpu_get_level");
        }
    }
}

}  // namespace ORB_SLAM2
