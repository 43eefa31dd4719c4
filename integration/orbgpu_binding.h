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
}  // namespace ORB_SLAM2
