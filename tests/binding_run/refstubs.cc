// tests/binding_run/refstubs.cc -- TEST-ONLY definitions of the reference-side members that the matcher and stereo
// drop-in bindings (integration/ORBmatcher_perframe.cc, integration/Frame_stereo.cc) read but do not define, over the
// restated declarations of integration/refdecl.  In ORB-SLAM2 these come from src/Frame.cc, src/MapPoint.cc,
// src/KeyFrame.cc and the part of src/ORBmatcher.cc the binding keeps (constructor, constants).  Not product code:
// tests/binding_run/run_matchers.cc links it to execute the bindings (tests/test_gpu_binding_matchers.py).
//
// The refdecl classes restate only the public members the bindings use, so the private state of MapPoint and
// KeyFrame (world position, descriptor, observations, distance bounds; the map-point matches) is kept in side tables
// keyed by the object.  The accessor bodies restate the reference's (file:line cited at each).
#include <cmath>
#include <cstring>
#include <unordered_map>

#include "ORBmatcher.h"
#include "refstubs.h"

namespace ORB_SLAM2 {

// src/ORBmatcher.cc:37-39, :41 (kept in the reference's ORBmatcher.cc next to the keyframe-rate overloads)
const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;
ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

// Frame's static calibration and grid geometry (include/Frame.h:116-119,167-168,191-194)
float Frame::fx, Frame::fy, Frame::cx, Frame::cy;
float Frame::mfGridElementWidthInv, Frame::mfGridElementHeightInv;
float Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY;

static std::unordered_map<const MapPoint*, MapPointState>& mp_state()
{
    static std::unordered_map<const MapPoint*, MapPointState> m;
    return m;
}
static std::unordered_map<const KeyFrame*, std::vector<MapPoint*>>& kf_matches()
{
    static std::unordered_map<const KeyFrame*, std::vector<MapPoint*>> m;
    return m;
}

MapPointState& state_of(const MapPoint* p) { return mp_state()[p]; }
void set_map_point_matches(const KeyFrame* kf, const std::vector<MapPoint*>& v) { kf_matches()[kf] = v; }

cv::Mat MapPoint::GetWorldPos()  // src/MapPoint.cc:80-84 (returns a copy)
{
    cv::Mat x(3, 1, CV_32F);
    for (int k = 0; k < 3; k++) x.at<float>(k) = state_of(this).pos[k];
    return x;
}
int MapPoint::Observations() { return state_of(this).nobs; }  // src/MapPoint.cc:145-149
bool MapPoint::isBad() { return state_of(this).bad; }         // src/MapPoint.cc:217-222
cv::Mat MapPoint::GetDescriptor()                             // src/MapPoint.cc:309-313 (a copy)
{
    cv::Mat d(1, 32, CV_8U);
    std::memcpy(d.data, state_of(this).desc, 32);
    return d;
}
float MapPoint::GetMinDistanceInvariance() { return 0.8f * state_of(this).min_dist; }  // src/MapPoint.cc:373-377
float MapPoint::GetMaxDistanceInvariance() { return 1.2f * state_of(this).max_dist; }  // src/MapPoint.cc:379-383
int MapPoint::PredictScale(const float& currentDist, Frame* pF)                         // src/MapPoint.cc:402-417
{
    const float ratio = state_of(this).max_dist / currentDist;
    int nScale = (int)std::ceil(std::log(ratio) / pF->mfLogScaleFactor);  // float log: `using namespace std`
    if (nScale < 0) nScale = 0;
    else if (nScale >= pF->mnScaleLevels) nScale = pF->mnScaleLevels - 1;
    return nScale;
}

std::vector<MapPoint*> KeyFrame::GetMapPointMatches() { return kf_matches()[this]; }  // src/KeyFrame.cc:283-287

}  // namespace ORB_SLAM2
