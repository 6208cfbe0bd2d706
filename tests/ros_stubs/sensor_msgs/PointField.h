// Test stand-in for sensor_msgs/PointField (tests/ros_stubs/README.md).
#pragma once
#include <cstdint>
#include <string>

namespace sensor_msgs {
struct PointField {
    std::string name;
    uint32_t offset = 0;
    uint8_t datatype = 0;
    uint32_t count = 1;
    static const uint8_t FLOAT32 = 7;
    static const uint8_t FLOAT64 = 8;
};
}  // namespace sensor_msgs
