// Test stand-in for geometry_msgs/PoseStamped (tests/ros_stubs/README.md).
#pragma once
#include <memory>

#include "../std_msgs/Header.h"

namespace geometry_msgs {
struct Point { double x = 0, y = 0, z = 0; };
struct Quaternion { double x = 0, y = 0, z = 0, w = 1; };
struct Pose {
    Point position;
    Quaternion orientation;
};
struct PoseStamped {
    std_msgs::Header header;
    Pose pose;
};
typedef std::shared_ptr<const PoseStamped> PoseStampedConstPtr;
}  // namespace geometry_msgs
