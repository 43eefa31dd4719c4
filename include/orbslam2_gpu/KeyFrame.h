/*
 * KeyFrame.h -- the part of ORB_SLAM2::KeyFrame (include/KeyFrame.h) that the relocalisation matcher
 * SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist) reads (src/ORBmatcher.cc:
 * 1472-1599): the undistorted keypoints and the map-point matches (GetMapPointMatches, include/KeyFrame.h).
 */
#ifndef ORBSLAM2_GPU_KEYFRAME_H
#define ORBSLAM2_GPU_KEYFRAME_H

#include <mutex>
#include <vector>

#include "MapPoint.h"
#include "Types.h"

namespace ORB_SLAM2
{

class KeyFrame
{
public:
    KeyFrame() = default;
    KeyFrame(const std::vector<KeyPoint>& keysUn, const std::vector<MapPoint*>& mapPoints)
        : mvKeysUn(keysUn), N((int)keysUn.size()), mvpMapPoints(mapPoints)
    {
    }

    std::vector<MapPoint*> GetMapPointMatches()
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        return mvpMapPoints;
    }

    const std::vector<KeyPoint> mvKeysUn;
    const int N = 0;

protected:
    std::vector<MapPoint*> mvpMapPoints;
    std::mutex mMutexFeatures;
};

}  // namespace ORB_SLAM2

#endif
