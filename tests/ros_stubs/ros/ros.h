// Test stand-in for roscpp (tests/ros_stubs/README.md): NodeHandle params (defaults, or
// "name=value;..." overrides from $TSDF_STUB_PARAMS), subscriptions by topic, and a spin() that
// replays $TSDF_STUB_STREAM (tsdf_replay's "TSDFSTR2" topic stream) into them in arrival order:
// 'P' records to the pose subscription, 'C' records (dlio::Point-shaped PointCloud2) to the cloud
// subscription, 'S' records call the node's advertised "save_map" service (~save_map), an 'X'
// record ends the process on the spot (a crash: no destructors run).
#pragma once
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../geometry_msgs/PoseStamped.h"
#include "../sensor_msgs/PointCloud2.h"
#include "../std_msgs/Header.h"

#define ROS_LOG_STUB_(lvl, ...)                   \
    do {                                          \
        std::fprintf(stderr, "[%s] ", lvl);       \
        std::fprintf(stderr, __VA_ARGS__);        \
        std::fprintf(stderr, "\n");               \
    } while (0)
#define ROS_INFO(...) ROS_LOG_STUB_("INFO", __VA_ARGS__)
#define ROS_WARN(...) ROS_LOG_STUB_("WARN", __VA_ARGS__)
#define ROS_ERROR(...) ROS_LOG_STUB_("ERROR", __VA_ARGS__)
#define ROS_FATAL(...) ROS_LOG_STUB_("FATAL", __VA_ARGS__)
#define ROS_WARN_THROTTLE(period, ...) ROS_LOG_STUB_("WARN", __VA_ARGS__)

namespace ros {

namespace stub {
// topic -> callback taking the message as shared_ptr<const void>
inline std::map<std::string, std::function<void(std::shared_ptr<const void>)>>& subs() {
    static std::map<std::string, std::function<void(std::shared_ptr<const void>)>> m;
    return m;
}
// service name (the private name as advertised) -> handler returning the response's success
inline std::map<std::string, std::function<bool()>>& services() {
    static std::map<std::string, std::function<bool()>> m;
    return m;
}
inline std::string param_override(const std::string& name) {
    const char* e = std::getenv("TSDF_STUB_PARAMS");
    if (!e) return "";
    std::stringstream ss(e);
    std::string kv;
    while (std::getline(ss, kv, ';')) {
        const size_t eq = kv.find('=');
        if (eq != std::string::npos && kv.substr(0, eq) == name) return kv.substr(eq + 1);
    }
    return "";
}
inline void parse(const std::string& s, double& v) { v = std::atof(s.c_str()); }
inline void parse(const std::string& s, int& v) { v = std::atoi(s.c_str()); }
inline void parse(const std::string& s, bool& v) { v = s == "1" || s == "true"; }
inline void parse(const std::string& s, std::string& v) { v = s; }
}  // namespace stub

class Subscriber {};
class ServiceServer {};

class NodeHandle {
   public:
    NodeHandle() {}
    explicit NodeHandle(const std::string&) {}
    template <class T>
    bool param(const std::string& name, T& v, const T& def) {
        const std::string o = stub::param_override(name);
        if (o.empty()) {
            v = def;
            return false;
        }
        stub::parse(o, v);
        return true;
    }
    template <class M, class C>
    Subscriber subscribe(const std::string& topic, uint32_t, void (C::*fn)(const std::shared_ptr<const M>&),
                         C* obj) {
        stub::subs()[topic] = [obj, fn](std::shared_ptr<const void> m) {
            (obj->*fn)(std::static_pointer_cast<const M>(m));
        };
        return Subscriber();
    }
    template <class Req, class Res, class C>
    ServiceServer advertiseService(const std::string& name, bool (C::*fn)(Req&, Res&), C* obj) {
        stub::services()[name] = [obj, fn, name]() {
            Req q;
            Res r;
            const bool ok = (obj->*fn)(q, r);
            std::fprintf(stderr, "[STUB] service %s: %s %s\n", name.c_str(),
                         ok && r.success ? "success" : "failure", r.message.c_str());
            return ok && r.success;
        };
        return ServiceServer();
    }
};

inline void init(int&, char**, const std::string&) {}
inline void shutdown() {}

// Replays $TSDF_STUB_STREAM into the subscriptions (cloud records as dlio::Point-shaped clouds:
// fields x, y, z float32 at offsets 0, 4, 8 of the record's point_step).
inline void spin() {
    const char* path = std::getenv("TSDF_STUB_STREAM");
    if (!path) return;
    FILE* f = std::fopen(path, "rb");
    if (!f) return;
    char magic[8];
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, "TSDFSTR2", 8) != 0) {
        std::fclose(f);
        return;
    }
    const std::string pose_topic = "robot/dlio/odom_node/pose";
    const std::string cloud_topic = "robot/dlio/odom_node/pointcloud/deskewed";
    for (;;) {
        char type = 0;
        int64_t t = 0;
        if (std::fread(&type, 1, 1, f) != 1 || std::fread(&t, 8, 1, f) != 1) break;
        if (type == 'P') {
            double v[7];
            if (std::fread(v, 8, 7, f) != 7) break;
            auto m = std::make_shared<geometry_msgs::PoseStamped>();
            m->header.stamp.ns = (uint64_t)t;
            m->pose.position.x = v[0];
            m->pose.position.y = v[1];
            m->pose.position.z = v[2];
            m->pose.orientation.x = v[3];
            m->pose.orientation.y = v[4];
            m->pose.orientation.z = v[5];
            m->pose.orientation.w = v[6];
            if (stub::subs().count(pose_topic)) stub::subs()[pose_topic](m);
        } else if (type == 'C') {
            uint64_t n = 0;
            uint32_t step = 0, xoff = 0;
            int32_t f64 = 0;
            if (std::fread(&n, 8, 1, f) != 1 || std::fread(&step, 4, 1, f) != 1 ||
                std::fread(&xoff, 4, 1, f) != 1 || std::fread(&f64, 4, 1, f) != 1)
                break;
            auto m = std::make_shared<sensor_msgs::PointCloud2>();
            m->header.stamp.ns = (uint64_t)t;
            m->width = (uint32_t)n;
            m->point_step = step;
            m->row_step = step * (uint32_t)n;
            const char* names[3] = {"x", "y", "z"};
            for (int k = 0; k < 3; k++) {
                sensor_msgs::PointField pf;
                pf.name = names[k];
                pf.offset = xoff + (f64 ? 8u : 4u) * (uint32_t)k;
                pf.datatype = f64 ? sensor_msgs::PointField::FLOAT64 : sensor_msgs::PointField::FLOAT32;
                m->fields.push_back(pf);
            }
            m->data.resize((size_t)n * step);
            if (n && std::fread(m->data.data(), step, n, f) != n) break;
            if (stub::subs().count(cloud_topic)) stub::subs()[cloud_topic](m);
        } else if (type == 'S') {  // a call of ~save_map at this point of the stream
            if (stub::services().count("save_map")) stub::services()["save_map"]();
        } else if (type == 'X') {  // the process dies here: no destructor, no shutdown save
            std::fflush(stderr);
            std::_Exit(3);
        } else {
            break;
        }
    }
    std::fclose(f);
}

}  // namespace ros
