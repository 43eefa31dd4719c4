/*
 * MapPoint.h -- the part of ORB_SLAM2::MapPoint (include/MapPoint.h, src/MapPoint.cc) that the per-frame
 * matchers read and that Frame::isInFrustum writes.
 *
 * Geometry (GetWorldPos, GetNormal, min/max distance), the representative descriptor, the observation
 * count and the bad flag are read under per-point mutexes as in the reference (src/MapPoint.cc:309-313,
 * 373-417); the matchers gather them into a structure-of-arrays snapshot at call time and hand that to
 * the GPU.  The tracking fields (mbTrackInView ... mTrackViewCos, include/MapPoint.h:91-99) are plain
 * members, as in the reference.
 */
#ifndef ORBSLAM2_GPU_MAPPOINT_H
#define ORBSLAM2_GPU_MAPPOINT_H

#include <array>
#include <cstring>
#include <mutex>

#include "Types.h"

namespace ORB_SLAM2
{

class MapPoint
{
public:
    MapPoint() = default;
    MapPoint(const float pos[3], const float normal[3], float minDistance, float maxDistance,
             const uint8_t descriptor[32], int nObs = 2)
    {
        SetWorldPos(pos);
        SetNormal(normal);
        SetDistances(minDistance, maxDistance);
        SetDescriptor(descriptor);
        SetObservations(nObs);
    }

    void SetWorldPos(const float p[3])
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        std::memcpy(mWorldPos.data(), p, sizeof(float) * 3);
    }
    std::array<float, 3> GetWorldPos()
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        return mWorldPos;
    }
    void SetNormal(const float n[3])
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        std::memcpy(mNormalVector.data(), n, sizeof(float) * 3);
    }
    std::array<float, 3> GetNormal()
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        return mNormalVector;
    }
    void SetDistances(float minDistance, float maxDistance)
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        mfMinDistance = minDistance;
        mfMaxDistance = maxDistance;
    }
    /* src/MapPoint.cc:373-383 return 0.8f*mfMinDistance and 1.2f*mfMaxDistance; isInFrustum reads those. */
    float GetMinDistanceInvariance()
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        return 0.8f * mfMinDistance;
    }
    float GetMaxDistanceInvariance()
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        return 1.2f * mfMaxDistance;
    }
    float MinDistanceRaw()
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        return mfMinDistance;
    }
    float MaxDistanceRaw()
    {
        std::lock_guard<std::mutex> lock(mMutexPos);
        return mfMaxDistance;
    }

    void SetDescriptor(const uint8_t d[32])
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        std::memcpy(mDescriptor.data(), d, 32);
    }
    std::array<uint8_t, 32> GetDescriptor()
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        return mDescriptor;
    }
    void SetObservations(int n)
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        nObs = n;
    }
    int Observations()
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        return nObs;
    }
    void SetBadFlag(bool bad = true)
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        mbBad = bad;
    }
    bool isBad()
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        return mbBad;
    }

    // Variables used by the tracking (include/MapPoint.h:91-99)
    float mTrackProjX = 0.f;
    float mTrackProjY = 0.f;
    float mTrackProjXR = 0.f;
    bool mbTrackInView = false;
    int mnTrackScaleLevel = 0;
    float mTrackViewCos = 0.f;

protected:
    std::array<float, 3> mWorldPos{};
    std::array<float, 3> mNormalVector{};
    float mfMinDistance = 0.f;
    float mfMaxDistance = 0.f;
    std::array<uint8_t, 32> mDescriptor{};
    int nObs = 0;
    bool mbBad = false;
    std::mutex mMutexPos;
    std::mutex mMutexFeatures;
};

}  // namespace ORB_SLAM2

#endif
