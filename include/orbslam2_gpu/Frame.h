/*
 * Frame.h -- ORB_SLAM2::Frame's per-frame feature path (include/Frame.h, src/Frame.cc) over the gfx950
 * C ABI.
 *
 * The three constructors run what the reference runs at frame creation, on the GPU: ORB extraction
 * (ExtractORB, both images concurrently for stereo as src/Frame.cc:78-81), UndistortKeyPoints,
 * ComputeStereoMatches / ComputeStereoFromRGBD, and the one-time ComputeImageBounds + grid scales.
 * AssignFeaturesToGrid's grid is built in HBM by the matchers (og_grid_kernel), so the host Frame keeps
 * no mGrid.  isInFrustum fills the MapPoint tracking fields (Frame::isInFrustum + MapPoint::
 * PredictScale); isInFrustum(points, ...) does the same for a whole local map in one launch, the form
 * Tracking::SearchLocalPoints should call (src/Tracking.cc:1167-1180).
 *
 * The static members (fx ... mnMaxY, grid scales, mbInitialComputations, nNextId) keep the reference's
 * process-wide semantics: they are set by the first frame (or after mbInitialComputations is reset).
 */
#ifndef ORBSLAM2_GPU_FRAME_H
#define ORBSLAM2_GPU_FRAME_H

#include <vector>

#include "KeyFrame.h"
#include "MapPoint.h"
#include "ORBVocabulary.h"
#include "ORBextractor.h"
#include "Types.h"

namespace ORB_SLAM2
{
#define FRAME_GRID_ROWS 48
#define FRAME_GRID_COLS 64

class Frame
{
public:
    Frame() = default;
    Frame(const Frame& frame) = default;

    // Constructor for stereo cameras (src/Frame.cc:61-123).
    Frame(const ImageU8& imLeft, const ImageU8& imRight, const double& timeStamp, ORBextractor* extractorLeft,
          ORBextractor* extractorRight, ORBVocabulary* voc, const CameraMatrix& K, const DistCoef& distCoef,
          const float& bf, const float& thDepth);

    // Constructor for RGB-D cameras (src/Frame.cc:125-175).
    Frame(const ImageU8& imGray, const DepthImage& imDepth, const double& timeStamp, ORBextractor* extractor,
          ORBVocabulary* voc, const CameraMatrix& K, const DistCoef& distCoef, const float& bf,
          const float& thDepth);

    // Constructor for Monocular cameras (src/Frame.cc:178-228).
    Frame(const ImageU8& imGray, const double& timeStamp, ORBextractor* extractor, ORBVocabulary* voc,
          const CameraMatrix& K, const DistCoef& distCoef, const float& bf, const float& thDepth);

    // Extract ORB on the image. 0 for left image and 1 for right image (src/Frame.cc:247-253).
    void ExtractORB(int flag, const ImageU8& im);

    // Compute Bag of Words representation (src/Frame.cc:395-402).
    void ComputeBoW();

    // Set the camera pose (src/Frame.cc:255-266).
    void SetPose(const Pose& Tcw);
    void UpdatePoseMatrices();
    std::array<float, 3> GetCameraCenter() const { return mOw; }

    // Check if a MapPoint is in the frustum of the camera and fill the MapPoint tracking variables
    // (src/Frame.cc:269-325).
    bool isInFrustum(MapPoint* pMP, float viewingCosLimit);
    // The same for every point of vpMapPoints in one GPU launch; returns the number in view.
    int isInFrustum(const std::vector<MapPoint*>& vpMapPoints, float viewingCosLimit);

    // Search a match for each keypoint in the left image to a keypoint in the right image
    // (src/Frame.cc:466-640; on the device pyramids of both extractors).
    void ComputeStereoMatches();

    // Associate a "right" coordinate to a keypoint if there is valid depth in the depthmap
    // (src/Frame.cc:643-664).
    void ComputeStereoFromRGBD(const DepthImage& imDepth);

    // Snapshot of the fields the GPU matchers read (mvKeysUn, mDescriptors, mvuRight, bounds, scales).
    orbgpu_frame_view view() const;
    orbgpu_camera camera() const;
    static orbgpu_grid_geom grid_geom();

public:
    ORBVocabulary* mpORBvocabulary = nullptr;
    ORBextractor* mpORBextractorLeft = nullptr;
    ORBextractor* mpORBextractorRight = nullptr;

    double mTimeStamp = 0.0;

    CameraMatrix mK;
    static float fx;
    static float fy;
    static float cx;
    static float cy;
    static float invfx;
    static float invfy;
    DistCoef mDistCoef;

    float mbf = 0.f;
    float mb = 0.f;
    float mThDepth = 0.f;

    int N = 0;

    std::vector<KeyPoint> mvKeys, mvKeysRight;
    std::vector<KeyPoint> mvKeysUn;

    std::vector<float> mvuRight;
    std::vector<float> mvDepth;

    DBoW2::BowVector mBowVec;
    DBoW2::FeatureVector mFeatVec;

    Descriptors mDescriptors, mDescriptorsRight;

    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;

    static float mfGridElementWidthInv;
    static float mfGridElementHeightInv;

    Pose mTcw;

    static long unsigned int nNextId;
    long unsigned int mnId = 0;

    KeyFrame* mpReferenceKF = nullptr;

    int mnScaleLevels = 0;
    float mfScaleFactor = 0.f;
    float mfLogScaleFactor = 0.f;
    std::vector<float> mvScaleFactors;
    std::vector<float> mvInvScaleFactors;
    std::vector<float> mvLevelSigma2;
    std::vector<float> mvInvLevelSigma2;

    static float mnMinX;
    static float mnMaxX;
    static float mnMinY;
    static float mnMaxY;

    static bool mbInitialComputations;

private:
    void InitScaleInfo(ORBextractor* extractor);
    void InitialComputations(const ImageU8& im, const CameraMatrix& K);
    void UndistortKeyPoints();
    void ComputeImageBounds(const ImageU8& imLeft);

    std::array<float, 9> mRcw{};
    std::array<float, 3> mtcw{};
    std::array<float, 9> mRwc{};
    std::array<float, 3> mOw{};
};

}  // namespace ORB_SLAM2

#endif
