/*
 * ORBextractor.h -- ORB_SLAM2::ORBextractor over the gfx950 C ABI (include/orbgpu.h).
 *
 * Mirrors the reference class include/ORBextractor.h:45-111: same constructor arguments, the same
 * operator() (mask ignored, empty image -> outputs untouched), the same inline getters and the public
 * mvImagePyramid member read by Frame::ComputeStereoMatches (src/Frame.cc:473,563,575,580).  One
 * instance owns one orbgpu context (its own HIP stream and device buffers), so two instances may run
 * concurrently from two threads as the stereo Frame constructor does (src/Frame.cc:78-81); one
 * instance is not re-entrant, as in the reference.
 */
#ifndef ORBSLAM2_GPU_ORBEXTRACTOR_H
#define ORBSLAM2_GPU_ORBEXTRACTOR_H

#include <vector>

#include "Types.h"

namespace ORB_SLAM2
{

class ORBextractor
{
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    /* include/ORBextractor.h:51-52 / src/ORBextractor.cc:410-470; `device` selects the HIP device.
     * Throws GpuError when no gfx950 device or library is available (there is no CPU fallback). */
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0);
    ~ORBextractor();
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    /* src/ORBextractor.cc:1043-1105.  Keypoints in level-0 coordinates, levels 0..nlevels-1 concatenated;
     * descriptors row i <-> keypoint i (released when no keypoint is found). */
    void operator()(const ImageU8& image, const ImageU8& mask, std::vector<KeyPoint>& keypoints,
                    Descriptors& descriptors);

    int GetLevels() const { return nlevels; }
    float GetScaleFactor() const { return (float)scaleFactor; }
    std::vector<float> GetScaleFactors() const { return mvScaleFactor; }
    std::vector<float> GetInverseScaleFactors() const { return mvInvScaleFactor; }
    std::vector<float> GetScaleSigmaSquares() const { return mvLevelSigma2; }
    std::vector<float> GetInverseScaleSigmaSquares() const { return mvInvLevelSigma2; }

    /* The image pyramid of the last call (include/ORBextractor.h:85).  Downloaded from HBM after every
     * call unless SetPyramidDownload(false): the GPU stereo matcher reads the device copy, so a stereo or
     * mono pipeline that never reads this member can skip the PCIe transfer. */
    std::vector<ImageU8> mvImagePyramid;
    void SetPyramidDownload(bool on) { mbDownloadPyramid = on; }

    /* The orbgpu context (HIP stream, device buffers) behind this instance. */
    orbgpu_ctx* context() const { return mCtx; }
    int GetFeaturesPerLevel(int level) const { return mnFeaturesPerLevel.at(level); }

protected:
    orbgpu_ctx* mCtx = nullptr;
    bool mbDownloadPyramid = true;

    int nfeatures;
    double scaleFactor;
    int nlevels;
    int iniThFAST;
    int minThFAST;

    std::vector<int> mnFeaturesPerLevel;
    std::vector<float> mvScaleFactor;
    std::vector<float> mvInvScaleFactor;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;
};

/* Raises GpuError with the context's message when rc != ORBGPU_OK. */
void orbgpu_throw_if(orbgpu_ctx* ctx, int rc, const char* what);

}  // namespace ORB_SLAM2

#endif
