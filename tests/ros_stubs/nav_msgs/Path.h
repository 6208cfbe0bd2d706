// Test stand-in for nav_msgs/Path (tests/ros_stubs/README.md).
#pragma once
#include <memory>
#include <vector>

#include "../geometry_msgs/PoseStamped.h"

namespace nav_msgs {
struct Path {
    std_msgs::Header header;
    std::vector<geometry_msgs::PoseStamped> poses;
};
typedef std::shared_ptr<const Path> PathConstPtr;
}  // namespace nav_msgs
