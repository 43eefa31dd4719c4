// Compile-check shim (see opencv2/core/core.hpp): the reference's include/ORBextractor.h includes <opencv/cv.h>.
#pragma once
#include "../opencv2/core/core.hpp"
