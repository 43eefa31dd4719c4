// ORB_SLAM2::ORBmatcher's per-frame matchers over the gfx950 C ABI -- include/orbslam2_gpu/ORBmatcher.h.
// Reference: src/ORBmatcher.cc:37-39 (constants), :45-137 (SearchByProjection(Frame&, MapPoints, th)),
// :405-520 (SearchForInitialization), :1328-1470 (SearchByProjection(Frame&, const Frame&, th, bMono)),
// :1472-1599 (SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist)), :1647-1663 (DescriptorDistance).
//
// Each method snapshots what the reference reads through the MapPoint / KeyFrame getters (under their
// mutexes), runs the matcher on the GPU, and writes the result back into the same mutable arguments the
// reference writes.  Map-point ownership crosses the C ABI as indices: `owner[i]` is the index of the
// map point that holds keypoint i (-1 == NULL); claims that existed before the call get indices past the
// candidate range, so they block exactly as the reference's `mvpMapPoints[i2]` checks do.
#include "orbslam2_gpu/ORBmatcher.h"

#include <cstring>

namespace ORB_SLAM2
{

const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

ORBmatcher::ORBmatcher(float nnratio, bool checkOri) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

int ORBmatcher::DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orbgpu_descriptor_distance(a, b); }

static orbgpu_ctx* ctx_of(const Frame& F)
{
    if (!F.mpORBextractorLeft) throw GpuError("ORBmatcher: the frame has no extractor (GPU context)");
    return F.mpORBextractorLeft->context();
}

int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize)
{
    vnMatches12 = std::vector<int>(F1.mvKeysUn.size(), -1);
    if (vbPrevMatched.size() < F1.mvKeysUn.size())
        throw GpuError("SearchForInitialization: vbPrevMatched has fewer entries than F1 keypoints");
    const orbgpu_frame_view v1 = F1.view(), v2 = F2.view();
    int nmatches = 0;
    static_assert(sizeof(Point2f) == 2 * sizeof(float), "Point2f layout");
    orbgpu_ctx* ctx = ctx_of(F2);
    orbgpu_throw_if(ctx,
                    orbgpu_search_for_initialization(ctx, &v1, &v2, mfNNratio, mbCheckOrientation ? 1 : 0,
                                                     reinterpret_cast<float*>(vbPrevMatched.data()),
                                                     vnMatches12.empty() ? nullptr : vnMatches12.data(), windowSize,
                                                     &nmatches),
                    "orbgpu_search_for_initialization");
    return nmatches;
}

int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th)
{
    const int M = (int)vpMapPoints.size();
    std::vector<uint8_t> inView(M), bad(M), desc(32 * (size_t)M);
    std::vector<int32_t> level(M), nObs(M), owner(F.N, -1), ownerObs(F.N, 0);
    std::vector<float> vc(M), px(M), py(M), pxr(M);
    for (int m = 0; m < M; ++m) {  // snapshot under the per-point mutexes
        MapPoint* p = vpMapPoints[m];
        inView[m] = p->mbTrackInView;
        bad[m] = p->isBad();
        level[m] = p->mnTrackScaleLevel;
        vc[m] = p->mTrackViewCos;
        px[m] = p->mTrackProjX;
        py[m] = p->mTrackProjY;
        pxr[m] = p->mTrackProjXR;
        nObs[m] = p->Observations();
        const auto d = p->GetDescriptor();
        std::memcpy(&desc[32 * (size_t)m], d.data(), 32);
    }
    for (int i = 0; i < F.N; ++i)  // existing claims (src/ORBmatcher.cc:87-89)
        if (F.mvpMapPoints[i]) {
            owner[i] = M;
            ownerObs[i] = F.mvpMapPoints[i]->Observations() > 0;
        }
    const orbgpu_frame_view v = F.view();
    orbgpu_mappoints_view mp{M, inView.data(), bad.data(), level.data(), vc.data(), px.data(), py.data(),
                             pxr.data(), nObs.data(), desc.data()};
    int nmatches = 0;
    orbgpu_ctx* ctx = ctx_of(F);
    orbgpu_throw_if(ctx,
                    orbgpu_search_by_projection(ctx, &v, &mp, mfNNratio, th, F.N ? owner.data() : nullptr,
                                                F.N ? ownerObs.data() : nullptr, &nmatches),
                    "orbgpu_search_by_projection");
    for (int i = 0; i < F.N; ++i)
        if (owner[i] >= 0 && owner[i] < M) F.mvpMapPoints[i] = vpMapPoints[owner[i]];
    return nmatches;
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono)
{
    const int n = LastFrame.N;
    std::vector<uint8_t> hasMp(n), outlier(n), desc(32 * (size_t)n);
    std::vector<float> pos(3 * (size_t)n);
    std::vector<int32_t> nObs(n);
    for (int i = 0; i < n; ++i) {
        MapPoint* p = LastFrame.mvpMapPoints[i];
        hasMp[i] = p != nullptr;
        outlier[i] = LastFrame.mvbOutlier[i];
        if (!p) continue;
        const auto P = p->GetWorldPos();
        for (int k = 0; k < 3; ++k) pos[3 * i + k] = P[k];
        nObs[i] = p->Observations();
        const auto d = p->GetDescriptor();
        std::memcpy(&desc[32 * (size_t)i], d.data(), 32);
    }
    const int N = CurrentFrame.N;
    std::vector<int32_t> owner(N, -1), ownerObs(N, 0);
    for (int i = 0; i < N; ++i)  // claims that exist before the call: indices n + i
        if (CurrentFrame.mvpMapPoints[i]) {
            owner[i] = n + i;
            ownerObs[i] = CurrentFrame.mvpMapPoints[i]->Observations() > 0;
        }
    const std::vector<MapPoint*> before = CurrentFrame.mvpMapPoints;
    orbgpu_last_frame_view lf{n,           reinterpret_cast<const orbgpu_keypoint*>(LastFrame.mvKeysUn.data()),
                              hasMp.data(), outlier.data(), pos.data(), nObs.data(), desc.data()};
    const orbgpu_frame_view v = CurrentFrame.view();
    const orbgpu_camera cur = CurrentFrame.camera(), last = LastFrame.camera();
    int nmatches = 0;
    orbgpu_ctx* ctx = ctx_of(CurrentFrame);
    orbgpu_throw_if(ctx,
                    orbgpu_search_by_projection_last_frame(ctx, &v, &cur, &last, &lf, th, bMono ? 1 : 0,
                                                           mbCheckOrientation ? 1 : 0, N ? owner.data() : nullptr,
                                                           N ? ownerObs.data() : nullptr, &nmatches),
                    "orbgpu_search_by_projection_last_frame");
    for (int i = 0; i < N; ++i) {
        const int o = owner[i];
        CurrentFrame.mvpMapPoints[i] = o < 0 ? nullptr : (o < n ? LastFrame.mvpMapPoints[o] : before[o - n]);
    }
    return nmatches;
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist)
{
    const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
    const int n = (int)vpMPs.size();
    if ((int)pKF->mvKeysUn.size() < n) throw GpuError("SearchByProjection(KeyFrame): fewer keypoints than matches");
    std::vector<uint8_t> valid(n), desc(32 * (size_t)n);
    std::vector<float> pos(3 * (size_t)n), mx(n), mn(n);
    for (int i = 0; i < n; ++i) {
        MapPoint* p = vpMPs[i];
        valid[i] = p && !p->isBad() && !sAlreadyFound.count(p);
        if (!valid[i]) continue;
        const auto P = p->GetWorldPos();
        for (int k = 0; k < 3; ++k) pos[3 * i + k] = P[k];
        mx[i] = p->MaxDistanceRaw();
        mn[i] = p->MinDistanceRaw();
        const auto d = p->GetDescriptor();
        std::memcpy(&desc[32 * (size_t)i], d.data(), 32);
    }
    const int N = CurrentFrame.N;
    std::vector<int32_t> owner(N, -1);
    for (int i = 0; i < N; ++i)
        if (CurrentFrame.mvpMapPoints[i]) owner[i] = n + i;  // any existing claim blocks (src/ORBmatcher.cc:1543)
    const std::vector<MapPoint*> before = CurrentFrame.mvpMapPoints;
    orbgpu_keyframe_view kf{n,          reinterpret_cast<const orbgpu_keypoint*>(pKF->mvKeysUn.data()),
                            valid.data(), pos.data(), mx.data(), mn.data(), desc.data()};
    const orbgpu_frame_view v = CurrentFrame.view();
    const orbgpu_camera cur = CurrentFrame.camera();
    int nmatches = 0;
    orbgpu_ctx* ctx = ctx_of(CurrentFrame);
    orbgpu_throw_if(ctx,
                    orbgpu_search_by_projection_keyframe(ctx, &v, &cur, &kf, th, ORBdist, mbCheckOrientation ? 1 : 0,
                                                         N ? owner.data() : nullptr, &nmatches),
                    "orbgpu_search_by_projection_keyframe");
    for (int i = 0; i < N; ++i) {
        const int o = owner[i];
        CurrentFrame.mvpMapPoints[i] = o < 0 ? nullptr : (o < n ? vpMPs[o] : before[o - n]);
    }
    return nmatches;
}

}  // namespace ORB_SLAM2
