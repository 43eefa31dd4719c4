// COMPILE-CHECK HEADER (see ORBmatcher.h in this directory): the KeyFrame declarations the binding reads.
#pragma once
#include <vector>

#include <opencv2/core/core.hpp>

namespace ORB_SLAM2 {
class MapPoint;
class KeyFrame
{
public:
    std::vector<MapPoint*> GetMapPointMatches();  // ref: include/KeyFrame.h:93
    const std::vector<cv::KeyPoint> mvKeysUn;  // ref: include/KeyFrame.h:170
};
}  // namespace ORB_SLAM2
