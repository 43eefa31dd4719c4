// integration/orbgpu_binding.h -- glue shared by the drop-in replacement sources of this directory.
//
// The replacement src/ORBextractor.cc keeps the reference's include/ORBextractor.h byte-identical: each extractor's
// gfx950 context lives in a side table keyed by the extractor (ORB-SLAM2 constructs its extractors once and never
// deletes them, src/Tracking.cc:119-125), so no member has to be added to the class.  The matcher and Frame
// replacements find the context of a Frame's extractor here.
#pragma once
#include "orbgpu.h"

namespace ORB_SLAM2 {
class ORBextractor;
// the context created for `ex` by the replacement ORBextractor constructor (nullptr if none)
orbgpu_ctx* orbgpu_context_of(const ORBextractor* ex);
// destroy the context of `ex` (for integrators that delete extractors; the reference never does)
void orbgpu_release_extractor(const ORBextractor* ex);
// refresh ex->mvImagePyramid after each call (on by default unless integration/Frame_stereo.cc is linked;
// ORBGPU_HOST_PYRAMID=0/1 sets the default)
void orbgpu_set_host_pyramid(const ORBextractor* ex, bool on);
}  // namespace ORB_SLAM2
