// Test stand-in for std_msgs/Header (tests/ros_stubs/README.md).
#pragma once
#include <cstdint>
#include <string>

namespace ros {
struct Time {
    uint64_t ns = 0;
    uint64_t toNSec() const { return ns; }
};
}  // namespace ros

namespace std_msgs {
struct Header {
    uint32_t seq = 0;
    ros::Time stamp;
    std::string frame_id;
};
}  // namespace std_msgs
