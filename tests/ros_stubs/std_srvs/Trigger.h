// Test stand-in for std_srvs/Trigger (tests/ros_stubs/README.md): an empty request, a response of
// (success, message) -- the fields the node's ~save_map service fills.
#pragma once
#include <string>

namespace std_srvs {
struct Trigger {
    struct Request {};
    struct Response {
        bool success = false;
        std::string message;
    };
    Request request;
    Response response;
};
}  // namespace std_srvs
