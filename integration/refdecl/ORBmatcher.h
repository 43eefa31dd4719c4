// integration/refdecl -- COMPILE-CHECK HEADERS (tests/test_integration_compile.py), not product code.
// The reference's include/Frame.h, MapPoint.h, KeyFrame.h and ORBmatcher.h pull in Eigen, g2o, DBoW2 and the
// quadric add-on, which this image lacks.  These headers restate ONLY the declarations the integration/ sources
// use; every restated line ends with `// ref: <file>:<line>` and the test checks that the reference header has that
// declaration at that line (whitespace-normalised), so the restatement cannot drift from the reference.
#pragma once
#include <set>
#include <utility>
#include <vector>

#include <opencv2/core/core.hpp>

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {
using std::pair;
using std::vector;

class ORBmatcher
{
public:
    ORBmatcher(float nnratio=0.6, bool checkOri=true);  // ref: include/ORBmatcher.h:41
    static int DescriptorDistance(const cv::Mat &a, const cv::Mat &b);  // ref: include/ORBmatcher.h:44
    int SearchByProjection(Frame &F, const std::vector<MapPoint*> &vpMapPoints, const float th=3);  // ref: include/ORBmatcher.h:48
    int SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, const float th, const bool bMono);  // ref: include/ORBmatcher.h:52
    int SearchByProjection(Frame &CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*> &sAlreadyFound, const float th, const int ORBdist);  // ref: include/ORBmatcher.h:56
    int SearchForInitialization(Frame &F1, Frame &F2, std::vector<cv::Point2f> &vbPrevMatched, std::vector<int> &vnMatches12, int windowSize=10);  // ref: include/ORBmatcher.h:69
    static const int TH_LOW;  // ref: include/ORBmatcher.h:87
    static const int TH_HIGH;  // ref: include/ORBmatcher.h:88
    static const int HISTO_LENGTH;  // ref: include/ORBmatcher.h:89
protected:
    float mfNNratio;  // ref: include/ORBmatcher.h:100
    bool mbCheckOrientation;  // ref: include/ORBmatcher.h:101
};
}  // namespace ORB_SLAM2
