// COMPILE-CHECK HEADER (see ORBmatcher.h in this directory): the Frame declarations the binding reads.
#pragma once
#include <vector>

#include <opencv2/core/core.hpp>

#include "MapPoint.h"
#include "ORBextractor.h"

namespace ORB_SLAM2 {
using std::vector;

class Frame
{
public:
    void ComputeStereoMatches();  // ref: include/Frame.h:96
    ORBextractor* mpORBextractorLeft, *mpORBextractorRight;  // ref: include/Frame.h:109
    static float fx;  // ref: include/Frame.h:116
    static float fy;  // ref: include/Frame.h:117
    static float cx;  // ref: include/Frame.h:118
    static float cy;  // ref: include/Frame.h:119
    float mbf;  // ref: include/Frame.h:125
    float mb;  // ref: include/Frame.h:128
    int N;  // ref: include/Frame.h:135
    std::vector<cv::KeyPoint> mvKeysUn;  // ref: include/Frame.h:143
    std::vector<float> mvuRight;    //float means sub_pixel  // ref: include/Frame.h:147
    std::vector<float> mvDepth;  // ref: include/Frame.h:148
    cv::Mat mDescriptors, mDescriptorsRight;  // ref: include/Frame.h:158
    std::vector<MapPoint*> mvpMapPoints;  // ref: include/Frame.h:161
    std::vector<bool> mvbOutlier;  // ref: include/Frame.h:164
    static float mfGridElementWidthInv;  // ref: include/Frame.h:167
    static float mfGridElementHeightInv;  // ref: include/Frame.h:168
    cv::Mat mTcw;  // ref: include/Frame.h:172
    int mnScaleLevels;  // ref: include/Frame.h:182
    float mfScaleFactor;  // ref: include/Frame.h:183
    float mfLogScaleFactor;  // ref: include/Frame.h:184
    vector<float> mvScaleFactors;  // ref: include/Frame.h:185
    static float mnMinX;  // ref: include/Frame.h:191
    static float mnMaxX;  // ref: include/Frame.h:192
    static float mnMinY;  // ref: include/Frame.h:193
    static float mnMaxY;  // ref: include/Frame.h:194
};
}  // namespace ORB_SLAM2
