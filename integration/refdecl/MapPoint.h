// COMPILE-CHECK HEADER (see ORBmatcher.h in this directory): the MapPoint declarations the binding reads.
#pragma once
#include <opencv2/core/core.hpp>

namespace ORB_SLAM2 {
class Frame;
class KeyFrame;
class MapPoint
{
public:
    cv::Mat GetWorldPos();  // ref: include/MapPoint.h:46
    int Observations();  // ref: include/MapPoint.h:52
    bool isBad();  // ref: include/MapPoint.h:61
    cv::Mat GetDescriptor();  // ref: include/MapPoint.h:75
    float GetMinDistanceInvariance();  // ref: include/MapPoint.h:79
    float GetMaxDistanceInvariance();  // ref: include/MapPoint.h:80
    int PredictScale(const float &currentDist, Frame* pF);  // ref: include/MapPoint.h:82
    float mTrackProjX;  // ref: include/MapPoint.h:92
    float mTrackProjY;  // ref: include/MapPoint.h:93
    float mTrackProjXR;  // ref: include/MapPoint.h:94
    bool mbTrackInView;  // ref: include/MapPoint.h:95
    int mnTrackScaleLevel;  // ref: include/MapPoint.h:96
    float mTrackViewCos;  // ref: include/MapPoint.h:97
};
}  // namespace ORB_SLAM2
