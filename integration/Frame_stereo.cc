// integration/Frame_stereo.cc -- Frame::ComputeStereoMatches (src/Frame.cc:466-640) on the gfx950 path: both
// extractors were just run on the rectified pair (src/Frame.cc:78-81), so their device pyramids, keypoints and
// descriptors are resident and the whole function is one call.  Replaces that body in src/Frame.cc.
#include <stdexcept>
#include <vector>

#include "Frame.h"
#include "orbgpu.h"
#include "orbgpu_binding.h"

// marks this replacement as linked: integration/ORBextractor.cc then skips the host pyramid download
extern "C" const int orbgpu_binding_device_stereo = 1;

namespace ORB_SLAM2 {

void Frame::ComputeStereoMatches()
{
    mvuRight = std::vector<float>(N, -1.0f);
    mvDepth = std::vector<float>(N, -1.0f);
    int n = 0, nmatches = 0;
    const int rc = orbgpu_compute_stereo_matches(orbgpu_context_of(mpORBextractorLeft),
                                                 orbgpu_context_of(mpORBextractorRight), mbf, mb, mvuRight.data(),
                                                 mvDepth.data(), N, &n, &nmatches);
    if (rc != ORBGPU_OK || n != N) throw std::runtime_error("orbgpu_compute_stereo_matches");
}

}  // namespace ORB_SLAM2
