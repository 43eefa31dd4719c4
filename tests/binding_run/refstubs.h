// tests/binding_run/refstubs.h -- side-table state of the test-only MapPoint / KeyFrame definitions
// (tests/binding_run/refstubs.cc).  Test infrastructure.
#pragma once
#include <cstdint>
#include <vector>

#include "KeyFrame.h"
#include "MapPoint.h"

namespace ORB_SLAM2 {
struct MapPointState {
    float pos[3] = {0, 0, 0};
    uint8_t desc[32] = {0};
    int nobs = 0;
    bool bad = false;
    float min_dist = 0, max_dist = 0;  // mfMinDistance / mfMaxDistance
};
MapPointState& state_of(const MapPoint* p);
void set_map_point_matches(const KeyFrame* kf, const std::vector<MapPoint*>& v);
}  // namespace ORB_SLAM2
