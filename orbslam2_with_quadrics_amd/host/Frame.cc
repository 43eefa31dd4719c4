// ORB_SLAM2::Frame's per-frame feature path over the gfx950 C ABI -- include/orbslam2_gpu/Frame.h.
// Reference: src/Frame.cc (constructors :61-228, ExtractORB :247-253, SetPose/UpdatePoseMatrices :255-266,
// isInFrustum :269-325, ComputeBoW :395-402, UndistortKeyPoints :404-434, ComputeImageBounds :436-461,
// ComputeStereoMatches :466-640, ComputeStereoFromRGBD :643-664).
#include "orbslam2_gpu/Frame.h"

#include <cmath>
#include <exception>
#include <thread>

namespace ORB_SLAM2
{

long unsigned int Frame::nNextId = 0;
bool Frame::mbInitialComputations = true;
float Frame::cx, Frame::cy, Frame::fx, Frame::fy, Frame::invfx, Frame::invfy;
float Frame::mnMinX, Frame::mnMinY, Frame::mnMaxX, Frame::mnMaxY;
float Frame::mfGridElementWidthInv, Frame::mfGridElementHeightInv;

namespace
{
bool distorted(const DistCoef& d) { return !d.empty() && d[0] != 0.0; }

// The extractor context also keeps mvKeysUn in HBM for the device-side consumers (RGB-D lookup, batched
// matchers); ndist == 0 switches that off (src/Frame.cc:406 copies mvKeys when k1 == 0).
void bind_undistortion(ORBextractor* ex, const CameraMatrix& K, const DistCoef& dist)
{
    const float K4[4] = {K.fx, K.fy, K.cx, K.cy};
    const int nd = distorted(dist) ? (int)dist.size() : 0;
    orbgpu_throw_if(ex->context(), orbgpu_set_undistortion(ex->context(), K4, nd ? dist.data() : nullptr, nd),
                    "orbgpu_set_undistortion");
}
}  // namespace

void Frame::InitScaleInfo(ORBextractor* extractor)
{
    mnScaleLevels = extractor->GetLevels();
    mfScaleFactor = extractor->GetScaleFactor();
    mfLogScaleFactor = std::log(mfScaleFactor);  // float log: `using namespace std`
    mvScaleFactors = extractor->GetScaleFactors();
    mvInvScaleFactors = extractor->GetInverseScaleFactors();
    mvLevelSigma2 = extractor->GetScaleSigmaSquares();
    mvInvLevelSigma2 = extractor->GetInverseScaleSigmaSquares();
}

void Frame::InitialComputations(const ImageU8& im, const CameraMatrix& K)
{
    // This is done only for the first Frame (or after a change in the calibration)
    if (mbInitialComputations) {
        ComputeImageBounds(im);
        mfGridElementWidthInv = static_cast<float>(FRAME_GRID_COLS) / static_cast<float>(mnMaxX - mnMinX);
        mfGridElementHeightInv = static_cast<float>(FRAME_GRID_ROWS) / static_cast<float>(mnMaxY - mnMinY);
        fx = K.fx;
        fy = K.fy;
        cx = K.cx;
        cy = K.cy;
        invfx = 1.0f / fx;
        invfy = 1.0f / fy;
        mbInitialComputations = false;
    }
    mb = mbf / fx;
}

// stereo: src/Frame.cc:61-123
Frame::Frame(const ImageU8& imLeft, const ImageU8& imRight, const double& timeStamp, ORBextractor* extractorLeft,
             ORBextractor* extractorRight, ORBVocabulary* voc, const CameraMatrix& K, const DistCoef& distCoef,
             const float& bf, const float& thDepth)
    : mpORBvocabulary(voc), mpORBextractorLeft(extractorLeft), mpORBextractorRight(extractorRight),
      mTimeStamp(timeStamp), mK(K), mDistCoef(distCoef), mbf(bf), mThDepth(thDepth)
{
    mnId = nNextId++;
    InitScaleInfo(mpORBextractorLeft);

    // ORB extraction: both extractors concurrently, each on its own context and HIP stream
    std::exception_ptr errLeft, errRight;
    std::thread threadLeft([&] {
        try {
            ExtractORB(0, imLeft);
        } catch (...) {
            errLeft = std::current_exception();
        }
    });
    std::thread threadRight([&] {
        try {
            ExtractORB(1, imRight);
        } catch (...) {
            errRight = std::current_exception();
        }
    });
    threadLeft.join();
    threadRight.join();
    if (errLeft) std::rethrow_exception(errLeft);
    if (errRight) std::rethrow_exception(errRight);

    N = (int)mvKeys.size();
    if (mvKeys.empty()) return;

    UndistortKeyPoints();
    // The reference reads mb (assigned mbf/fx only further down) inside ComputeStereoMatches
    // (minZ = mb, maxD = mbf/minZ); the value it is meant to hold is used here.
    mb = mbf / (mbInitialComputations ? K.fx : fx);
    ComputeStereoMatches();

    mvpMapPoints = std::vector<MapPoint*>(N, static_cast<MapPoint*>(nullptr));
    mvbOutlier = std::vector<bool>(N, false);
    InitialComputations(imLeft, K);
}

// RGB-D: src/Frame.cc:125-175
Frame::Frame(const ImageU8& imGray, const DepthImage& imDepth, const double& timeStamp, ORBextractor* extractor,
             ORBVocabulary* voc, const CameraMatrix& K, const DistCoef& distCoef, const float& bf,
             const float& thDepth)
    : mpORBvocabulary(voc), mpORBextractorLeft(extractor), mpORBextractorRight(nullptr), mTimeStamp(timeStamp),
      mK(K), mDistCoef(distCoef), mbf(bf), mThDepth(thDepth)
{
    mnId = nNextId++;
    InitScaleInfo(mpORBextractorLeft);
    bind_undistortion(mpORBextractorLeft, mK, mDistCoef);  // mvKeysUn on the device for the depth lookup
    ExtractORB(0, imGray);
    N = (int)mvKeys.size();
    if (mvKeys.empty()) return;
    UndistortKeyPoints();
    ComputeStereoFromRGBD(imDepth);
    mvpMapPoints = std::vector<MapPoint*>(N, static_cast<MapPoint*>(nullptr));
    mvbOutlier = std::vector<bool>(N, false);
    InitialComputations(imGray, K);
}

// monocular: src/Frame.cc:178-228
Frame::Frame(const ImageU8& imGray, const double& timeStamp, ORBextractor* extractor, ORBVocabulary* voc,
             const CameraMatrix& K, const DistCoef& distCoef, const float& bf, const float& thDepth)
    : mpORBvocabulary(voc), mpORBextractorLeft(extractor), mpORBextractorRight(nullptr), mTimeStamp(timeStamp),
      mK(K), mDistCoef(distCoef), mbf(bf), mThDepth(thDepth)
{
    mnId = nNextId++;
    InitScaleInfo(mpORBextractorLeft);
    ExtractORB(0, imGray);
    N = (int)mvKeys.size();
    if (mvKeys.empty()) return;
    UndistortKeyPoints();
    // Set no stereo information
    mvuRight = std::vector<float>(N, -1);
    mvDepth = std::vector<float>(N, -1);
    mvpMapPoints = std::vector<MapPoint*>(N, static_cast<MapPoint*>(nullptr));
    mvbOutlier = std::vector<bool>(N, false);
    InitialComputations(imGray, K);
}

void Frame::ExtractORB(int flag, const ImageU8& im)
{
    if (flag == 0)
        (*mpORBextractorLeft)(im, ImageU8(), mvKeys, mDescriptors);
    else
        (*mpORBextractorRight)(im, ImageU8(), mvKeysRight, mDescriptorsRight);
}

void Frame::SetPose(const Pose& Tcw)
{
    mTcw = Tcw;
    mTcw.empty = false;
    UpdatePoseMatrices();
}

void Frame::UpdatePoseMatrices()
{
    const float* T = mTcw.T;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) {
            mRcw[3 * r + c] = T[4 * r + c];
            mRwc[3 * c + r] = T[4 * r + c];
        }
        mtcw[r] = T[4 * r + 3];
    }
    // mOw = -mRcw.t()*mtcw: cv::Mat's 3-term float product sum, then alpha = -1 (this file
    // is compiled with -ffp-contract=off, as OpenCV's baseline build has no FMA)
    for (int r = 0; r < 3; ++r) {
        const float s = (mRwc[3 * r] * mtcw[0] + mRwc[3 * r + 1] * mtcw[1]) + mRwc[3 * r + 2] * mtcw[2];
        mOw[r] = (float)((double)s * -1.0);
    }
}

orbgpu_grid_geom Frame::grid_geom()
{
    orbgpu_grid_geom g;
    g.minX = mnMinX;
    g.minY = mnMinY;
    g.maxX = mnMaxX;
    g.maxY = mnMaxY;
    g.invW = mfGridElementWidthInv;
    g.invH = mfGridElementHeightInv;
    return g;
}

orbgpu_frame_view Frame::view() const
{
    orbgpu_frame_view v;
    v.n = N;
    v.kps = reinterpret_cast<const orbgpu_keypoint*>(mvKeysUn.data());
    v.desc = mDescriptors.data();
    v.uright = mvuRight.empty() ? nullptr : mvuRight.data();
    v.grid = grid_geom();
    v.scale_factors = mvScaleFactors.data();
    v.nlevels = (int)mvScaleFactors.size();
    return v;
}

orbgpu_camera Frame::camera() const
{
    orbgpu_camera c;
    for (int i = 0; i < 9; ++i) c.Rcw[i] = mRcw[i];
    for (int i = 0; i < 3; ++i) {
        c.tcw[i] = mtcw[i];
        c.Ow[i] = mOw[i];
    }
    c.fx = fx;
    c.fy = fy;
    c.cx = cx;
    c.cy = cy;
    c.mbf = mbf;
    c.mb = mb;
    c.scale_factor = mfScaleFactor;
    c.nlevels = mnScaleLevels;
    return c;
}

int Frame::isInFrustum(const std::vector<MapPoint*>& vpMapPoints, float viewingCosLimit)
{
    const int m = (int)vpMapPoints.size();
    if (m == 0) return 0;
    std::vector<float> pos(3 * (size_t)m), nrm(3 * (size_t)m), mx(m), mn(m);
    for (int i = 0; i < m; ++i) {  // snapshot under the per-point mutexes
        MapPoint* p = vpMapPoints[i];
        const auto P = p->GetWorldPos();
        const auto Nn = p->GetNormal();
        for (int k = 0; k < 3; ++k) {
            pos[3 * i + k] = P[k];
            nrm[3 * i + k] = Nn[k];
        }
        mx[i] = p->MaxDistanceRaw();
        mn[i] = p->MinDistanceRaw();
    }
    orbgpu_mappoint_geom_view g{m, pos.data(), nrm.data(), mx.data(), mn.data()};
    std::vector<uint8_t> inView(m);
    std::vector<float> px(m), py(m), pxr(m), vc(m);
    std::vector<int32_t> level(m);
    int nIn = 0;
    const orbgpu_camera cam = camera();
    orbgpu_ctx* ctx = mpORBextractorLeft->context();
    orbgpu_throw_if(ctx,
                    orbgpu_is_in_frustum(ctx, &cam, grid_geom(), &g, viewingCosLimit, inView.data(), px.data(),
                                         py.data(), pxr.data(), level.data(), vc.data(), &nIn),
                    "orbgpu_is_in_frustum");
    for (int i = 0; i < m; ++i) {
        MapPoint* p = vpMapPoints[i];
        p->mbTrackInView = inView[i] != 0;
        if (!inView[i]) continue;
        p->mTrackProjX = px[i];
        p->mTrackProjXR = pxr[i];
        p->mTrackProjY = py[i];
        p->mnTrackScaleLevel = level[i];
        p->mTrackViewCos = vc[i];
    }
    return nIn;
}

bool Frame::isInFrustum(MapPoint* pMP, float viewingCosLimit)
{
    return isInFrustum(std::vector<MapPoint*>{pMP}, viewingCosLimit) == 1;
}

void Frame::ComputeBoW()
{
    if (mBowVec.empty())
        mpORBvocabulary->transform(mpORBextractorLeft->context(), mDescriptors, mBowVec, mFeatVec, 4);
}

void Frame::UndistortKeyPoints()
{
    if (!distorted(mDistCoef)) {
        mvKeysUn = mvKeys;
        return;
    }
    const float K4[4] = {mK.fx, mK.fy, mK.cx, mK.cy};
    mvKeysUn.resize(N);
    orbgpu_ctx* ctx = mpORBextractorLeft->context();
    orbgpu_throw_if(ctx,
                    orbgpu_undistort_keypoints(ctx, K4, mDistCoef.data(), (int)mDistCoef.size(),
                                               reinterpret_cast<const orbgpu_keypoint*>(mvKeys.data()),
                                               reinterpret_cast<orbgpu_keypoint*>(mvKeysUn.data()), N),
                    "orbgpu_undistort_keypoints");
}

void Frame::ComputeImageBounds(const ImageU8& imLeft)
{
    if (distorted(mDistCoef)) {
        const float K4[4] = {mK.fx, mK.fy, mK.cx, mK.cy};
        orbgpu_grid_geom g;
        orbgpu_ctx* ctx = mpORBextractorLeft->context();
        orbgpu_throw_if(ctx,
                        orbgpu_compute_image_bounds(ctx, K4, mDistCoef.data(), (int)mDistCoef.size(), imLeft.cols,
                                                    imLeft.rows, &g),
                        "orbgpu_compute_image_bounds");
        mnMinX = g.minX;
        mnMaxX = g.maxX;
        mnMinY = g.minY;
        mnMaxY = g.maxY;
    } else {
        mnMinX = 0.0f;
        mnMaxX = imLeft.cols;
        mnMinY = 0.0f;
        mnMaxY = imLeft.rows;
    }
}

void Frame::ComputeStereoMatches()
{
    mvuRight.assign(N, -1.0f);
    mvDepth.assign(N, -1.0f);
    int n = 0, nm = 0;
    orbgpu_ctx* ctx = mpORBextractorLeft->context();
    orbgpu_throw_if(ctx,
                    orbgpu_compute_stereo_matches(ctx, mpORBextractorRight->context(), mbf, mb, mvuRight.data(),
                                                  mvDepth.data(), N, &n, &nm),
                    "orbgpu_compute_stereo_matches");
    if (n != N) throw GpuError("orbgpu_compute_stereo_matches: keypoint count mismatch");
}

void Frame::ComputeStereoFromRGBD(const DepthImage& imDepth)
{
    mvuRight.assign(N, -1);
    mvDepth.assign(N, -1);
    int n = 0;
    orbgpu_ctx* ctx = mpORBextractorLeft->context();
    orbgpu_throw_if(ctx,
                    orbgpu_compute_stereo_from_rgbd(ctx, imDepth.data, imDepth.is_u16 ? 1 : 0, imDepth.factor,
                                                    imDepth.step, mbf, mvuRight.data(), mvDepth.data(), N, &n),
                    "orbgpu_compute_stereo_from_rgbd");
    if (n != N) throw GpuError("orbgpu_compute_stereo_from_rgbd: keypoint count mismatch");
}

}  // namespace ORB_SLAM2
