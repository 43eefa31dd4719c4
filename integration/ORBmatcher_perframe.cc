// integration/ORBmatcher_perframe.cc -- the per-frame ORBmatcher methods on the gfx950 path.
//
// A maintainer deletes these bodies from the reference's src/ORBmatcher.cc and adds this file; the keyframe-rate
// overloads (SearchByBoW, SearchByProjection(pKF, Scw, ..), SearchForTriangulation, SearchBySim3, Fuse) keep their
// CPU bodies there.  Signatures are the reference's
// (include/ORBmatcher.h:40-69); tests/test_integration_compile.py compiles this file against the restated
// declarations of integration/refdecl (checked line by line against the reference headers).
#include <cstdint>
#include <set>
#include <stdexcept>
#include <vector>

#include "ORBmatcher.h"
#include "orbgpu.h"
#include "orbgpu_binding.h"

namespace ORB_SLAM2 {

// A snapshot of the Frame fields the matchers read (mvKeysUn, mDescriptors, mvuRight, the static grid geometry)
static orbgpu_frame_view view_of(const Frame& F)
{
    orbgpu_frame_view v;
    v.n = F.N;
    v.kps = reinterpret_cast<const orbgpu_keypoint*>(F.mvKeysUn.data());
    v.desc = F.mDescriptors.data;  // N x 32, continuous
    v.uright = F.mvuRight.empty() ? nullptr : F.mvuRight.data();
    v.grid = orbgpu_grid_geom{Frame::mnMinX, Frame::mnMinY, Frame::mnMaxX, Frame::mnMaxY, Frame::mfGridElementWidthInv,
                              Frame::mfGridElementHeightInv};
    v.scale_factors = F.mvScaleFactors.data();
    v.nlevels = (int)F.mvScaleFactors.size();
    return v;
}

// Pose and intrinsics of a Frame; mOw = -Rcw^T tcw in float, as Frame::UpdatePoseMatrices computes it
// (src/Frame.cc:258-266; built without contraction, like OpenCV's own matrix code)
static orbgpu_camera camera_of(const Frame& F)
{
    orbgpu_camera c{};
    for (int r = 0; r < 3; ++r) {
        for (int k = 0; k < 3; ++k) c.Rcw[3 * r + k] = F.mTcw.at<float>(r, k);
        c.tcw[r] = F.mTcw.at<float>(r, 3);
    }
    for (int k = 0; k < 3; ++k)
        c.Ow[k] = -((c.Rcw[k] * c.tcw[0] + c.Rcw[3 + k] * c.tcw[1]) + c.Rcw[6 + k] * c.tcw[2]);
    c.fx = Frame::fx;
    c.fy = Frame::fy;
    c.cx = Frame::cx;
    c.cy = Frame::cy;
    c.mbf = F.mbf;
    c.mb = F.mb;
    c.scale_factor = F.mfScaleFactor;
    c.nlevels = F.mnScaleLevels;
    return c;
}

static orbgpu_ctx* ctx_of(const Frame& F)
{
    orbgpu_ctx* c = orbgpu_context_of(F.mpORBextractorLeft);
    if (!c) throw std::runtime_error("frame extractor has no gfx950 context (integration/ORBextractor.cc)");
    return c;
}

// src/ORBmatcher.cc:1647-1663 (host popcount of the same 8 words)
int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b)
{
    return orbgpu_descriptor_distance(a.ptr<uint8_t>(), b.ptr<uint8_t>());
}

// src/ORBmatcher.cc:405-520, called from Tracking::MonocularInitialization (src/Tracking.cc:599-600)
int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize)
{
    orbgpu_frame_view v1 = view_of(F1), v2 = view_of(F2);
    vnMatches12.assign(F1.mvKeysUn.size(), -1);
    int nmatches = 0;
    if (orbgpu_search_for_initialization(ctx_of(F2), &v1, &v2, mfNNratio, mbCheckOrientation,
                                         reinterpret_cast<float*>(vbPrevMatched.data()), vnMatches12.data(),
                                         windowSize, &nmatches) != ORBGPU_OK)
        throw std::runtime_error("orbgpu_search_for_initialization");
    return nmatches;
}

// src/ORBmatcher.cc:45-129, called from Tracking::SearchLocalPoints (src/Tracking.cc:1184-1191)
int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th)
{
    const int M = (int)vpMapPoints.size();
    std::vector<uint8_t> inView(M), bad(M), desc(32 * (size_t)M);
    std::vector<int32_t> level(M), nObs(M), owner(F.N, -1), ownerObs(F.N, 0);
    std::vector<float> vc(M), px(M), py(M), pxr(M);
    for (int m = 0; m < M; ++m) {  // snapshot through the per-point mutex getters
        MapPoint* p = vpMapPoints[m];
        inView[m] = p->mbTrackInView;
        bad[m] = p->isBad();
        level[m] = p->mnTrackScaleLevel;
        vc[m] = p->mTrackViewCos;
        px[m] = p->mTrackProjX;
        py[m] = p->mTrackProjY;
        pxr[m] = p->mTrackProjXR;
        nObs[m] = p->Observations();
        cv::Mat d(1, 32, CV_8U, &desc[32 * (size_t)m]);
        p->GetDescriptor().copyTo(d);
    }
    for (int i = 0; i < F.N; ++i)  // claims made before the call (src/ORBmatcher.cc:87-89)
        if (MapPoint* q = F.mvpMapPoints[i]) {
            owner[i] = M;
            ownerObs[i] = q->Observations() > 0;
        }
    orbgpu_frame_view v = view_of(F);
    orbgpu_mappoints_view mp{M, inView.data(), bad.data(), level.data(), vc.data(), px.data(), py.data(),
                             pxr.data(), nObs.data(), desc.data()};
    int nmatches = 0;
    if (orbgpu_search_by_projection(ctx_of(F), &v, &mp, mfNNratio, th, owner.data(), ownerObs.data(), &nmatches) !=
        ORBGPU_OK)
        throw std::runtime_error("orbgpu_search_by_projection");
    for (int i = 0; i < F.N; ++i)
        if (owner[i] >= 0 && owner[i] < M) F.mvpMapPoints[i] = vpMapPoints[owner[i]];
    return nmatches;
}

// src/ORBmatcher.cc:1328-1470, called from Tracking::TrackWithMotionModel (src/Tracking.cc:869-891)
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono)
{
    const int L = LastFrame.N;
    std::vector<uint8_t> has(L), outl(L), desc(32 * (size_t)L);
    std::vector<float> pos(3 * (size_t)L);
    std::vector<int32_t> nobs(L), owner(CurrentFrame.N, -1), ownerObs(CurrentFrame.N, 0);
    for (int i = 0; i < L; ++i) {
        MapPoint* p = LastFrame.mvpMapPoints[i];
        has[i] = p != nullptr;
        outl[i] = LastFrame.mvbOutlier[i];
        if (!p) continue;
        cv::Mat x = p->GetWorldPos();
        for (int k = 0; k < 3; ++k) pos[3 * i + k] = x.at<float>(k);
        nobs[i] = p->Observations();
        cv::Mat d(1, 32, CV_8U, &desc[32 * (size_t)i]);
        p->GetDescriptor().copyTo(d);
    }
    for (int i = 0; i < CurrentFrame.N; ++i)  // claims made before the call: L + i keeps the holder recoverable
        if (MapPoint* q = CurrentFrame.mvpMapPoints[i]) {
            owner[i] = L + i;
            ownerObs[i] = q->Observations() > 0;
        }
    const std::vector<MapPoint*> before = CurrentFrame.mvpMapPoints;
    orbgpu_last_frame_view lf{L, reinterpret_cast<const orbgpu_keypoint*>(LastFrame.mvKeysUn.data()), has.data(),
                              outl.data(), pos.data(), nobs.data(), desc.data()};
    orbgpu_frame_view v = view_of(CurrentFrame);
    orbgpu_camera cur = camera_of(CurrentFrame), last = camera_of(LastFrame);
    int nmatches = 0;
    if (orbgpu_search_by_projection_last_frame(ctx_of(CurrentFrame), &v, &cur, &last, &lf, th, bMono,
                                               mbCheckOrientation, owner.data(), ownerObs.data(),
                                               &nmatches) != ORBGPU_OK)
        throw std::runtime_error("orbgpu_search_by_projection_last_frame");
    // an owner of -1 is a keypoint the rotation check cleared (:1448-1467, mvpMapPoints[..] = NULL), even one that was
    // held before the call and taken over by a point with no observations
    for (int i = 0; i < CurrentFrame.N; ++i) {
        const int o = owner[i];
        CurrentFrame.mvpMapPoints[i] = o < 0 ? nullptr : (o < L ? LastFrame.mvpMapPoints[o] : before[o - L]);
    }
    return nmatches;
}

// src/ORBmatcher.cc:1472-1599, called from Tracking::Relocalization (src/Tracking.cc:1433,1467).  mfMaxDistance /
// mfMinDistance are protected (include/MapPoint.h:141-142), so the scale gate runs here with the point's own public
// methods -- GetMin/MaxDistanceInvariance and PredictScale on dist3D = cv::norm(x3Dw - Ow), exactly the reference's
// :1477-1523 -- and the projection, window search, claims and rotation histogram run on the GPU
// (orbgpu_search_by_projection_keyframe_levels).
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist)
{
    const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);
    const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
    const cv::Mat Ow = -Rcw.t() * tcw;
    const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
    const int L = (int)vpMPs.size();
    std::vector<uint8_t> valid(L, 0), desc(32 * (size_t)L, 0);
    std::vector<float> pos(3 * (size_t)L, 0.f);
    std::vector<int32_t> level(L, -1), owner(CurrentFrame.N, -1);
    for (int i = 0; i < L; ++i) {
        MapPoint* pMP = vpMPs[i];
        if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;
        valid[i] = 1;
        const cv::Mat x3Dw = pMP->GetWorldPos();
        for (int k = 0; k < 3; ++k) pos[3 * i + k] = x3Dw.at<float>(k);
        cv::Mat d(1, 32, CV_8U, &desc[32 * (size_t)i]);
        pMP->GetDescriptor().copyTo(d);
        const cv::Mat PO = x3Dw - Ow;
        const float dist3D = cv::norm(PO);
        const float maxDistance = pMP->GetMaxDistanceInvariance();
        const float minDistance = pMP->GetMinDistanceInvariance();
        if (dist3D < minDistance || dist3D > maxDistance) continue;  // level stays -1
        level[i] = pMP->PredictScale(dist3D, &CurrentFrame);
    }
    for (int i = 0; i < CurrentFrame.N; ++i)  // any claim blocks the keypoint (:1532-1533); L + i keeps the holder
        if (CurrentFrame.mvpMapPoints[i]) owner[i] = L + i;
    const std::vector<MapPoint*> before = CurrentFrame.mvpMapPoints;
    orbgpu_keyframe_view kf{L, reinterpret_cast<const orbgpu_keypoint*>(pKF->mvKeysUn.data()), valid.data(),
                            pos.data(), nullptr, nullptr, desc.data()};
    orbgpu_frame_view v = view_of(CurrentFrame);
    orbgpu_camera cur = camera_of(CurrentFrame);
    int nmatches = 0;
    if (orbgpu_search_by_projection_keyframe_levels(ctx_of(CurrentFrame), &v, &cur, &kf, level.data(), th, ORBdist,
                                                    mbCheckOrientation, owner.data(), &nmatches) != ORBGPU_OK)
        throw std::runtime_error("orbgpu_search_by_projection_keyframe_levels");
    // -1: cleared by the rotation check (:1577-1596) or never matched
    for (int i = 0; i < CurrentFrame.N; ++i) {
        const int o = owner[i];
        CurrentFrame.mvpMapPoints[i] = o < 0 ? nullptr : (o < L ? vpMPs[o] : before[o - L]);
    }
    return nmatches;
}

}  // namespace ORB_SLAM2
