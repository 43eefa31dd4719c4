// COMPILE-CHECK HEADER (see ORBmatcher.h in this directory).
#pragma once
namespace ORB_SLAM2 {
class KeyFrame;
}
