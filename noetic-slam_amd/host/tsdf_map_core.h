// tsdf_map_core.h — the ROS-free core of tsdf_map_node (MAP_BACKEND_IDX = 4): pose-track pairing
// of DLIO's clouds and the per-scan integrate call.  Shared by the ROS1 node
// (noetic-slam_amd/ros/tsdf_map_node.cpp) and the headless driver (host/tsdf_replay.cpp), so the
// node's logic is what the tests run.
//
// Pose pairing (the C++ twin of tsdf_map/ingest.py PoseTrack): DLIO stamps the
// deskewed cloud with the scan time (reference src/dlio/src/dlio/odom.cc:447) but publishes /pose at
// the IMU rate stamped with imu_stamp (odom.cc:318,383).  A cloud's ray origin is therefore the pose
// track evaluated at the cloud's stamp: linear interpolation of the position between the bracketing
// samples and slerp of the orientation (the sensor axes: Voxblox's 1/z^2 weight), the exact sample
// when a stamp matches; the scan goes to tsdf_integrate_pose.  A cloud newer than the newest pose
// waits (bounded queue) until the track passes its stamp; a cloud older than the track or across a
// gap wider than max_gap_ms is dropped and counted.  /path (nav_msgs/Path, appended per scan,
// odom.cc:358-432) can feed the same track.
//
// No copy of the cloud is made here: a waiting cloud is held by a reference to the caller's
// message (a shared_ptr keep-alive, e.g. the ROS ConstPtr), and tsdf_integrate_pose itself copies
// the points into pinned staging before it returns.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <vector>

#include "../../include/tsdf_hip.h"

namespace tsdf_map {

struct Pose {
    int64_t t_ns;
    double p[3];
    double q[4];  // x y z w
};

class PoseTrack {
   public:
    explicit PoseTrack(double keep_s = 10.0) : keep_ns_((int64_t)(keep_s * 1e9)) {}

    // Samples arrive in any order; kept sorted; samples older than keep_s behind the newest go.
    void add(const Pose& s) {
        auto it = std::upper_bound(v_.begin(), v_.end(), s.t_ns,
                                   [](int64_t t, const Pose& a) { return t < a.t_ns; });
        v_.insert(it, s);
        while (v_.size() > 2 && v_.back().t_ns - v_.front().t_ns > keep_ns_) v_.pop_front();
    }
    bool empty() const { return v_.empty(); }
    int64_t newest() const { return v_.empty() ? INT64_MIN : v_.back().t_ns; }
    int64_t oldest() const { return v_.empty() ? INT64_MAX : v_.front().t_ns; }

    // Pose at t_ns as (x, y, z, qx, qy, qz, qw) (ingest.py PoseTrack.at, the same double ops:
    // linear position, slerp orientation); false outside the track or across a gap wider than
    // max_gap_ms.
    bool at(int64_t t_ns, double max_gap_ms, double out[7]) const {
        if (v_.empty() || t_ns < v_.front().t_ns || t_ns > v_.back().t_ns) return false;
        auto it = std::lower_bound(v_.begin(), v_.end(), t_ns,
                                   [](const Pose& a, int64_t t) { return a.t_ns < t; });
        if (it->t_ns == t_ns) {
            std::memcpy(out, it->p, sizeof it->p);
            std::memcpy(out + 3, it->q, sizeof it->q);
            return true;
        }
        const Pose& b = *it;
        const Pose& a = *(it - 1);
        if ((double)(b.t_ns - a.t_ns) > max_gap_ms * 1e6) return false;
        const double f = (double)(t_ns - a.t_ns) / (double)(b.t_ns - a.t_ns);
        for (int k = 0; k < 3; k++) out[k] = a.p[k] + f * (b.p[k] - a.p[k]);
        slerp(a.q, b.q, f, out + 3);
        return true;
    }

    // ingest.py _slerp: shortest arc, normalised lerp above a dot of 0.9995
    static void slerp(const double q0[4], const double q1_in[4], double f, double out[4]) {
        double q1[4], d = 0.0;
        for (int k = 0; k < 4; k++) d += q0[k] * q1_in[k];
        const double s = d < 0.0 ? -1.0 : 1.0;
        for (int k = 0; k < 4; k++) q1[k] = s * q1_in[k];
        d *= s;
        if (d > 0.9995) {
            for (int k = 0; k < 4; k++) out[k] = q0[k] + f * (q1[k] - q0[k]);
        } else {
            const double th = std::acos(d);
            const double a = std::sin((1.0 - f) * th), b = std::sin(f * th), c = std::sin(th);
            for (int k = 0; k < 4; k++) out[k] = (a * q0[k] + b * q1[k]) / c;
        }
        double n = 0.0;
        for (int k = 0; k < 4; k++) n += out[k] * out[k];
        n = std::sqrt(n);
        for (int k = 0; k < 4; k++) out[k] /= n;
    }

   private:
    int64_t keep_ns_;
    std::deque<Pose> v_;
};

// The node's per-scan slot: clouds paired with the pose track, integrated through the C-ABI.
// One context, or N azimuth-sector contexts of tsdf_create_sharded (the node's ~num_gpus): each
// cloud then goes to all of them through tsdf_integrate_sectors (packed once, fanned out GPU to
// GPU; every context keeps its sector's rays).
class MapCore {
   public:
    struct Counts {
        uint64_t integrated = 0, dropped_old = 0, dropped_gap = 0, dropped_queue = 0;
    };

    MapCore(tsdf_ctx* ctx, double max_gap_ms = 50.0, size_t max_pending = 16)
        : ctxs_(1, ctx), max_gap_ms_(max_gap_ms), max_pending_(max_pending) {}
    MapCore(std::vector<tsdf_ctx*> ctxs, double max_gap_ms = 50.0, size_t max_pending = 16)
        : ctxs_(std::move(ctxs)), max_gap_ms_(max_gap_ms), max_pending_(max_pending) {}

    // A pose sample (PoseStamped / Odometry / a Path entry); releases the clouds it covers.
    int on_pose(const Pose& s) {
        track_.add(s);
        return release(false);
    }

    // One PointCloud2 payload.  `keep` owns the bytes at `data` (the message): it is held while the
    // cloud waits for its pose and released once the library has copied the points.
    int on_cloud(int64_t stamp_ns, std::shared_ptr<const void> keep, const void* data, uint64_t n,
                 uint32_t point_step, uint32_t xyz_offset, int32_t xyz_is_f64) {
        Pending c;
        c.t_ns = stamp_ns;
        c.n = n;
        c.step = point_step;
        c.xoff = xyz_offset;
        c.f64 = xyz_is_f64;
        c.keep = std::move(keep);
        c.data = data;
        pending_.push_back(std::move(c));
        if (pending_.size() > max_pending_) {  // the pose stream stalled: oldest cloud goes
            pending_.pop_front();
            counts_.dropped_queue++;
        }
        return release(false);
    }

    // End of stream: pair what can be paired with the track as it is.
    int flush() { return release(true); }

    const Counts& counts() const { return counts_; }
    size_t pending() const { return pending_.size(); }

   private:
    struct Pending {
        int64_t t_ns;
        uint64_t n;
        uint32_t step, xoff;
        int32_t f64;
        std::shared_ptr<const void> keep;  // the message owning `data`
        const void* data;
    };

    int release(bool final_) {
        while (!pending_.empty()) {
            Pending& c = pending_.front();
            if (!final_ && !track_.empty() && c.t_ns > track_.newest()) break;  // wait for poses
            if (!final_ && track_.empty()) break;
            double pose[7];
            if (!track_.at(c.t_ns, max_gap_ms_, pose)) {
                if (c.t_ns < track_.oldest() || track_.empty() || c.t_ns > track_.newest())
                    counts_.dropped_old++;
                else
                    counts_.dropped_gap++;
                pending_.pop_front();
                continue;
            }
            const int rc =
                ctxs_.size() == 1
                    ? tsdf_integrate_pose(ctxs_[0], c.data, c.n, c.step, c.xoff, c.f64, pose)
                    : tsdf_integrate_sectors(ctxs_.data(), (uint32_t)ctxs_.size(), c.data, c.n,
                                             c.step, c.xoff, c.f64, pose);
            pending_.pop_front();
            if (rc != TSDF_OK) return rc;
            counts_.integrated++;
        }
        return TSDF_OK;
    }

    std::vector<tsdf_ctx*> ctxs_;
    double max_gap_ms_;
    size_t max_pending_;
    PoseTrack track_;
    std::deque<Pending> pending_;
    Counts counts_;
};

}  // namespace tsdf_map
