"""MI355X-native ORB-SLAM2 feature hot path (ORB extraction + Hamming matching) -- drop-in for
yxqc/ORBSLAM2_with_quadrics's ORBextractor / ORBmatcher.

The compute path is the gfx950 HIP library liborbgpu.so (C ABI: include/orbgpu.h); these modules
are thin mirrors of the reference C++ classes for Python callers, tests and the bench.
"""
from .extractor import KP_DTYPE, ORBextractor  # noqa: F401
from .matcher import (ComputeImageBounds, ComputeStereoFromRGBD, ComputeStereoMatches, Frame, ORBmatcher,  # noqa: F401
                      UndistortKeyPoints)
from .vocabulary import ComputeBoW, ORBVocabulary  # noqa: F401

__all__ = ["ORBextractor", "ORBmatcher", "Frame", "ComputeStereoMatches", "UndistortKeyPoints", "ComputeImageBounds",
           "ComputeStereoFromRGBD", "ORBVocabulary", "ComputeBoW", "KP_DTYPE"]
