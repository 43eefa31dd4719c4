/*
 * ORBmatcher.h -- ORB_SLAM2::ORBmatcher's per-frame matchers (include/ORBmatcher.h:37-102) over the gfx950
 * C ABI.  Same constructor, same method signatures (OpenCV types replaced as in Types.h), same outputs
 * through the mutable Frame& / vector& arguments and the same returned match counts.  The keyframe-rate
 * matchers (SearchByBoW, SearchForTriangulation, SearchBySim3, Fuse, the Sim3 projection) are outside the
 * per-frame path and are not part of this layer.
 */
#ifndef ORBSLAM2_GPU_ORBMATCHER_H
#define ORBSLAM2_GPU_ORBMATCHER_H

#include <set>
#include <vector>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "Types.h"

namespace ORB_SLAM2
{

class ORBmatcher
{
public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true);

    // Computes the Hamming distance between two ORB descriptors (src/ORBmatcher.cc:1647-1663).
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b);

    // Search matches between Frame keypoints and projected MapPoints (src/ORBmatcher.cc:45-137).
    int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3);

    // Project MapPoints tracked in last frame into the current frame (src/ORBmatcher.cc:1328-1470).
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);

    // Project MapPoints seen in KeyFrame into the Frame (relocalisation, src/ORBmatcher.cc:1472-1599).
    int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                           const float th, const int ORBdist);

    // Matching for the Map Initialization (src/ORBmatcher.cc:405-520).
    int SearchForInitialization(Frame& F1, Frame& F2, std::vector<Point2f>& vbPrevMatched,
                                std::vector<int>& vnMatches12, int windowSize = 10);

public:
    static const int TH_LOW;
    static const int TH_HIGH;
    static const int HISTO_LENGTH;

protected:
    float mfNNratio;
    bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2

#endif
