// tsdf_map_node — the reference's TSDF mapping node (README.md:44-50) with the MI355X backend,
// MAP_BACKEND_IDX = 4.  ROS1 noetic; built by this directory's CMakeLists.txt inside a catkin
// workspace only (it needs roscpp, sensor_msgs, geometry_msgs, nav_msgs; nothing else of ROS is
// used, and no PCL: the PointCloud2 bytes go to the library as they arrive).
//
// Subscriptions (the reference's topic names, launch/dlio.launch:15-38):
//   ~cloud_topic  robot/dlio/odom_node/pointcloud/deskewed  sensor_msgs/PointCloud2 (dlio::Point,
//                 world frame; the slot of Dliomapping_Node::callback_pcl_deskewed,
//                 src/dliomapping/dliomapping.cpp:44,64-81)
//   ~pose_topic   robot/dlio/odom_node/pose                 geometry_msgs/PoseStamped (100 Hz,
//                 stamped with imu_stamp, src/dlio/src/dlio/odom.cc:318,383)
//   ~path_topic   (optional) robot/dlio/odom_node/path      nav_msgs/Path (per scan, odom.cc:358-432)
// Each cloud's ray origin is the pose track at the cloud's stamp (odom.cc:447), interpolated —
// tsdf_map::MapCore (host/tsdf_map_core.h), the object the headless driver host/tsdf_replay runs in
// the tests (tests/test_host_replay.py::test_topic_stream_*), so the pairing shipped here is the one
// tested.  Clouds newer than the newest pose wait for it.
//
// On shutdown the map is written like dliomapping's destructor writes its PLY (dliomapping.cpp:53-61):
// ~map_path (bricks: u64 n, i32 coords[3 n], f32 sdf[512 n], f32 weight[512 n]) and, with
// ~mesh_path set, a binary PLY triangle soup from tsdf_extract_mesh_table with ~mesh_table
// ("lorensen", the default: the published Lorensen / Bourke table VDBFusion's and voxblox's
// marching cubes compile in; "generated": this library's face-consistent table).
// Checkpoints while running: every ~save_every_n_clouds clouds (default 999, dliomapping's
// periodic PLY dump, dliomapping.cpp:72-80; 0: off) the map is written again, and the ~save_map
// service (std_srvs/Trigger; in the spirit of DLIO's save_pcd service, map.cc:81-111) writes the map
// and mesh on demand.  Every write goes to a temporary file renamed over ~map_path, so a crash
// mid-write keeps the previous checkpoint.
//
// Several GPUs (north_star: "scans shard by azimuth sector across up to 8 GPUs"; SURVEY §5's
// ~num_gpus): ~num_gpus = N > 1 creates N sector contexts with tsdf_create_sharded on ~device_ids
// ("0,1,2,3"; default 0 .. N-1) from ~sector_yaw0, each cloud goes to all of them through
// tsdf_integrate_sectors (packed once, one H2D copy, xGMI copies to the others, each GPU keeps its
// azimuth sector), and before the map or mesh is written tsdf_border_reduce_local moves every border
// brick's mass to one owner; the map file then holds every observed brick once and the mesh is
// tsdf_extract_mesh_local's (a one-brick halo exchanged between the GPUs, each cube meshed once).
// ~sector_rule: "index" (default, ABI v10: GPU k takes the k-th contiguous 1/N of every cloud's
// points -- DLIO's cloud is time-sorted, odom.cc:635-636, so a column range of the spin; each GPU
// receives only its share) or "world" (world-frame azimuth sectors from ~sector_yaw0).  If the
// border reduce fails (it is a transaction: the contexts are then unchanged), it is retried once,
// and then the map is written from every context's bricks merged on the host (the reduce's
// weighted mean) and the mesh from that merged map, so no session's map is lost to it.
#include <geometry_msgs/PoseStamped.h>
#include <nav_msgs/Path.h>
#include <ros/ros.h>
#include <sensor_msgs/PointCloud2.h>
#include <sensor_msgs/PointField.h>
#include <std_srvs/Trigger.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/tsdf_hip.h"
#include "../host/tsdf_map_core.h"

namespace {

tsdf_map::Pose to_pose(const std_msgs::Header& h, const geometry_msgs::Pose& p) {
    tsdf_map::Pose s;
    s.t_ns = (int64_t)h.stamp.toNSec();
    s.p[0] = p.position.x;
    s.p[1] = p.position.y;
    s.p[2] = p.position.z;
    s.q[0] = p.orientation.x;
    s.q[1] = p.orientation.y;
    s.q[2] = p.orientation.z;
    s.q[3] = p.orientation.w;
    return s;
}

class TsdfMapNode {
   public:
    explicit TsdfMapNode(ros::NodeHandle& nh, ros::NodeHandle& pnh) {
        tsdf_params p;
        tsdf_default_params(&p);  // 5 cm voxels, 15 cm truncation, no carving
        pnh.param("voxel_size", p.voxel_size, 0.05);
        pnh.param("sdf_trunc", p.sdf_trunc, 0.15);
        bool carving = false;
        pnh.param("space_carving", carving, false);
        p.space_carving = carving ? 1 : 0;
        pnh.param("min_range", p.min_range, 1.0);  // DLIO already crops +-1 m (odom.cc:490-526)
        int max_batch = 8, device = 0, pipeline = 0;
        pnh.param("max_batch", max_batch, max_batch);  // scans per GPU batch (latency vs rate)
        pnh.param("device_id", device, device);
        pnh.param("pipeline", pipeline, pipeline);
        p.max_batch = (uint32_t)max_batch;
        p.device_id = device;
        p.pipeline = (uint32_t)pipeline;
        int max_bricks = 1 << 20;
        pnh.param("max_bricks", max_bricks, max_bricks);  // initial pool; grows on demand
        p.max_bricks = (uint64_t)max_bricks;
        std::string sem;  // default: VDBFusion at upstream's own precisions
        pnh.param<std::string>("semantics", sem, "vdbfusion_f64");
        if (sem == "voxblox") {  // backend idx 2's rule
            p.semantics = TSDF_SEM_VOXBLOX;
            pnh.param("max_ray_length_m", p.max_range, 5.0);
            double mw = 10000.0;
            pnh.param("max_weight", mw, mw);
            p.max_weight = (float)mw;
            bool clear = true, drop = true, const_w = false;  // voxblox's Config defaults
            pnh.param("allow_clear", clear, clear);
            pnh.param("use_weight_dropoff", drop, drop);
            pnh.param("use_const_weight", const_w, const_w);  // false: 1 / z^2 (the pose's z axis)
            p.allow_clear = clear ? 1 : 0;
            p.use_weight_dropoff = drop ? 1 : 0;
            p.depth_weight = const_w ? 0 : 1;
            // voxblox_ros TsdfServer `method`: "merged" (its default) or "simple"
            std::string method;
            pnh.param<std::string>("method", method, "merged");
            if (method == "merged") {
                p.voxblox_method = TSDF_VB_MERGED;
            } else if (method == "simple") {
                p.voxblox_method = TSDF_VB_SIMPLE;
            } else {  // "fast" is thread-order dependent
                ROS_FATAL("unknown voxblox method '%s' (merged, simple)", method.c_str());
                ros::shutdown();
                return;
            }
        } else if (sem == "vdbfusion_f64") {  // upstream's precisions
            p.semantics = TSDF_SEM_VDBFUSION_F64;
        } else if (sem == "vdbfusion") {  // the fp32 restatement
            p.semantics = TSDF_SEM_VDBFUSION;
        } else {
            ROS_FATAL("unknown semantics '%s' (vdbfusion_f64, vdbfusion, voxblox)", sem.c_str());
            ros::shutdown();
            return;
        }
        // ~num_gpus sector contexts (one per GPU of ~device_ids), or one context on ~device_id
        int num_gpus = 1;
        pnh.param("num_gpus", num_gpus, num_gpus);
        std::string ids;
        pnh.param<std::string>("device_ids", ids, "");
        pnh.param("sector_yaw0", p.sector_yaw0, 0.0);
        std::string rule;
        pnh.param<std::string>("sector_rule", rule, "index");
        if (rule == "index") {
            p.sector_rule = TSDF_SECTOR_RULE_INDEX;
        } else if (rule == "world") {
            p.sector_rule = TSDF_SECTOR_RULE_WORLD;
        } else {
            ROS_FATAL("unknown sector_rule '%s' (index, world)", rule.c_str());
            ros::shutdown();
            return;
        }
        if (num_gpus < 1 || num_gpus > TSDF_MAX_WORLD) {
            ROS_FATAL("num_gpus must be 1 .. %d", TSDF_MAX_WORLD);
            ros::shutdown();
            return;
        }
        std::vector<int32_t> dev_ids;
        {
            std::stringstream ss(ids);
            std::string tok;
            while (std::getline(ss, tok, ',')) dev_ids.push_back((int32_t)std::atoi(tok.c_str()));
        }
        if (dev_ids.empty())
            for (int k = 0; k < num_gpus; k++) dev_ids.push_back(num_gpus == 1 ? device : k);
        if ((int)dev_ids.size() != num_gpus) {
            ROS_FATAL("device_ids lists %zu devices for num_gpus %d", dev_ids.size(), num_gpus);
            ros::shutdown();
            return;
        }
        ctxs_.assign((size_t)num_gpus, nullptr);
        const int crc = num_gpus == 1
                            ? (p.device_id = dev_ids[0], tsdf_create(&p, &ctxs_[0]))
                            : tsdf_create_sharded(&p, (uint32_t)num_gpus, dev_ids.data(), ctxs_.data());
        if (crc != TSDF_OK) {
            ROS_FATAL("tsdf_create%s failed (see stderr)", num_gpus > 1 ? "_sharded" : "");
            ctxs_.clear();
            ros::shutdown();
            return;
        }
        ctx_ = ctxs_[0];
        params_ = p;
        double max_gap_ms = 50.0;
        pnh.param("max_pose_gap_ms", max_gap_ms, max_gap_ms);
        core_ = new tsdf_map::MapCore(ctxs_, max_gap_ms);
        std::string metrics;
        pnh.param<std::string>("metrics_log", metrics, "");
        if (!metrics.empty() && tsdf_set_metrics_log(ctx_, metrics.c_str()) != TSDF_OK)
            ROS_WARN("metrics log: %s", tsdf_last_error(ctx_));
        pnh.param<std::string>("map_path", map_path_, "tsdf_map.bricks");
        pnh.param("save_every_n_clouds", save_every_, save_every_);
        pnh.param<std::string>("mesh_path", mesh_path_, "");
        std::string table;
        pnh.param<std::string>("mesh_table", table, "lorensen");
        if (table == "lorensen") {
            mesh_table_ = TSDF_MC_LORENSEN;
        } else if (table == "generated") {
            mesh_table_ = TSDF_MC_GENERATED;
        } else {
            ROS_FATAL("unknown mesh_table '%s' (lorensen, generated)", table.c_str());
            ros::shutdown();
            return;
        }
        std::string cloud_topic, pose_topic, path_topic;
        pnh.param<std::string>("cloud_topic", cloud_topic, "robot/dlio/odom_node/pointcloud/deskewed");
        pnh.param<std::string>("pose_topic", pose_topic, "robot/dlio/odom_node/pose");
        pnh.param<std::string>("path_topic", path_topic, "");
        sub_pose_ = nh.subscribe(pose_topic, 1000, &TsdfMapNode::on_pose, this);
        if (!path_topic.empty()) sub_path_ = nh.subscribe(path_topic, 10, &TsdfMapNode::on_path, this);
        sub_cloud_ = nh.subscribe(cloud_topic, 100, &TsdfMapNode::on_cloud, this);
        srv_save_ = pnh.advertiseService("save_map", &TsdfMapNode::on_save_map, this);
    }

    ~TsdfMapNode() {
        if (!ctx_) return;
        core_->flush();
        save(true);
        delete core_;
        for (tsdf_ctx* c : ctxs_) tsdf_destroy(c);
    }

    void on_pose(const geometry_msgs::PoseStampedConstPtr& m) {
        check(core_->on_pose(to_pose(m->header, m->pose)), "integrate");
    }

    void on_path(const nav_msgs::PathConstPtr& m) {
        if (m->poses.empty()) return;
        const auto& last = m->poses.back();  // /path grows by one pose per scan
        check(core_->on_pose(to_pose(last.header, last.pose)), "integrate");
    }

    // replaces Dliomapping_Node::callback_pcl_deskewed (dliomapping.cpp:64-81): no fromROSMsg,
    // the library reads x, y, z where the message says they are
    void on_cloud(const sensor_msgs::PointCloud2ConstPtr& msg) {
        int xoff = -1, f64 = 0;
        for (const auto& f : msg->fields)
            if (f.name == "x") {
                xoff = (int)f.offset;
                f64 = f.datatype == sensor_msgs::PointField::FLOAT64;
            }
        if (xoff < 0 || msg->is_bigendian) {
            ROS_WARN_THROTTLE(5.0, "cloud without little-endian x, y, z: skipped");
            return;
        }
        const uint64_t n = (uint64_t)msg->width * msg->height;
        // no copy: MapCore holds the message itself while the cloud waits for its pose (the
        // deleter keeps a reference to the ConstPtr), and the library copies the points once,
        // into pinned staging
        std::shared_ptr<const void> keep(msg.get(), [m = msg](const void*) mutable { m.reset(); });
        check(core_->on_cloud((int64_t)msg->header.stamp.toNSec(), std::move(keep), msg->data.data(),
                              n, msg->point_step, (uint32_t)xoff, f64),
              "integrate");
        // dliomapping's periodic dump (dliomapping.cpp:72-80): a checkpoint of the map so far
        if (save_every_ > 0 && ++clouds_ % (uint64_t)save_every_ == 0) {
            ROS_INFO("checkpoint after %llu clouds (%llu integrated)", (unsigned long long)clouds_,
                     (unsigned long long)core_->counts().integrated);
            save(false);
        }
    }

    // ~save_map: the map (and the mesh, with ~mesh_path) written now (DLIO's save_pcd, map.cc:81-111)
    bool on_save_map(std_srvs::Trigger::Request&, std_srvs::Trigger::Response& res) {
        ROS_INFO("save_map: %llu clouds integrated", (unsigned long long)core_->counts().integrated);
        res.success = save(true);
        res.message = res.success ? "saved " + map_path_ : "saving the map failed (see the log)";
        return true;
    }

   private:
    void check(int rc, const char* what) {
        if (rc != TSDF_OK) ROS_ERROR("tsdf %s: %s", what, tsdf_last_error(ctx_));
    }

    // One map: every context's bricks, each observed brick once.  With several GPUs the border
    // reduce runs first (retried once); if it still fails, the contexts are unchanged (the reduce
    // is a transaction) and their border bricks are merged here instead, in context order, by
    // the reduce's rule: S = (S_a W_a + S_b W_b) / (W_a + W_b), W = W_a + W_b, capped at max_weight
    // under Voxblox semantics (a voxel unobserved on one side is copied from the other).  Returns false when nothing could be read out.
    bool collect(std::vector<int32_t>& c, std::vector<float>& s, std::vector<float>& w,
                 bool& reduced) {
        const uint32_t n = (uint32_t)ctxs_.size();
        reduced = true;
        if (n > 1) {
            uint64_t moved = 0;
            int rc = tsdf_border_reduce_local(ctxs_.data(), n, &moved);
            if (rc != TSDF_OK) {
                ROS_WARN("tsdf border reduce: %s; retrying", tsdf_last_error(ctx_));
                rc = tsdf_border_reduce_local(ctxs_.data(), n, &moved);
            }
            if (rc != TSDF_OK) {
                ROS_ERROR("tsdf border reduce failed again (%s): merging the GPUs' bricks on the host",
                          tsdf_last_error(ctx_));
                reduced = false;
            } else {
                ROS_INFO("border reduce: %llu bricks moved", (unsigned long long)moved);
            }
        }
        std::unordered_map<uint64_t, uint64_t> at;  // brick key -> row (host merge only)
        // the reduce's weight cap: Voxblox's max_weight, none otherwise (tsdf_border_merge_device)
        const float w_cap = params_.semantics == TSDF_SEM_VOXBLOX ? params_.max_weight : INFINITY;
        for (tsdf_ctx* k : ctxs_) {
            uint64_t nb = 0, got = 0;
            if (tsdf_num_bricks(k, &nb) != TSDF_OK) return false;
            std::vector<int32_t> ck(3 * nb);
            std::vector<float> sk(512 * nb), wk(512 * nb);
            if (tsdf_export_bricks(k, ck.data(), sk.data(), wk.data(), nb, &got) != TSDF_OK) return false;
            for (uint64_t b = 0; b < got; b++) {
                const float* sb = sk.data() + 512 * b;
                const float* wb = wk.data() + 512 * b;
                bool obs = false;
                for (int l = 0; l < 512 && !obs; l++) obs = wb[l] > 0.0f;
                if (n > 1 && !obs) continue;
                if (!reduced) {
                    const uint64_t key = ((uint64_t)(uint32_t)(ck[3 * b] + (1 << 20)) << 42) |
                                         ((uint64_t)(uint32_t)(ck[3 * b + 1] + (1 << 20)) << 21) |
                                         (uint64_t)(uint32_t)(ck[3 * b + 2] + (1 << 20));
                    const auto it = at.find(key);
                    if (it != at.end()) {  // a border brick another context holds too: merge
                        float* so = s.data() + 512 * it->second;
                        float* wo = w.data() + 512 * it->second;
                        for (int l = 0; l < 512; l++) {
                            if (!(wb[l] > 0.0f)) continue;
                            if (!(wo[l] > 0.0f)) {
                                so[l] = sb[l];
                                wo[l] = wb[l];
                                continue;
                            }
                            const float wt = wo[l] + wb[l];
                            so[l] = (so[l] * wo[l] + sb[l] * wb[l]) / wt;
                            wo[l] = wt > w_cap ? w_cap : wt;
                        }
                        continue;
                    }
                    at.emplace(key, c.size() / 3);
                }
                c.insert(c.end(), ck.begin() + 3 * b, ck.begin() + 3 * b + 3);
                s.insert(s.end(), sb, sb + 512);
                w.insert(w.end(), wb, wb + 512);
            }
        }
        return true;
    }

    // The map (and, with_mesh and ~mesh_path, the mesh), each written to a temporary file and
    // renamed over the previous one.
    bool save(bool with_mesh) {
        const uint32_t n = (uint32_t)ctxs_.size();
        std::vector<int32_t> c;
        std::vector<float> s, w;
        bool reduced = true;
        if (!collect(c, s, w, reduced)) {
            ROS_ERROR("tsdf map read-out: %s", tsdf_last_error(ctx_));
            return false;
        }
        const uint64_t got = c.size() / 3;
        const std::string tmp = map_path_ + ".tmp";
        FILE* f = std::fopen(tmp.c_str(), "wb");
        bool ok = f != nullptr;
        if (f) {
            ok = std::fwrite(&got, 8, 1, f) == 1 && std::fwrite(c.data(), 4, 3 * got, f) == 3 * got &&
                 std::fwrite(s.data(), 4, 512 * got, f) == 512 * got &&
                 std::fwrite(w.data(), 4, 512 * got, f) == 512 * got;
            ok = std::fclose(f) == 0 && ok;
            ok = ok && std::rename(tmp.c_str(), map_path_.c_str()) == 0;
        }
        if (!ok) {
            ROS_ERROR("writing %s failed", map_path_.c_str());
            return false;
        }
        ROS_INFO("saved %llu bricks to %s%s", (unsigned long long)got, map_path_.c_str(),
                 reduced ? "" : " (host-merged)");
        if (!with_mesh || mesh_path_.empty()) return true;
        // the mesh of the reduced contexts or -- after a failed reduce -- of the host-merged map,
        // imported into a temporary context on the first GPU
        tsdf_ctx* tc = nullptr;
        if (!reduced) {
            tsdf_params q = params_;
            q.n_sectors = 0;
            q.sector = 0;
            q.max_bricks = std::max<uint64_t>(got, 1024);
            q.max_bricks_hard = 0;
            if (tsdf_create(&q, &tc) != TSDF_OK ||
                tsdf_import_bricks(tc, c.data(), s.data(), w.data(), got) != TSDF_OK) {
                ROS_ERROR("mesh of the host-merged map: %s", tc ? tsdf_last_error(tc) : "create failed");
                tsdf_destroy(tc);
                return false;
            }
        }
        auto mesh = [&](float* tri, uint64_t cap, uint64_t* nt) {
            if (tc) return tsdf_extract_mesh_table(tc, 0.0f, mesh_table_, tri, cap, nt);
            return n > 1 ? tsdf_extract_mesh_local(ctxs_.data(), n, 0.0f, mesh_table_, tri, cap, nt)
                         : tsdf_extract_mesh_table(ctx_, 0.0f, mesh_table_, tri, cap, nt);
        };
        uint64_t nt = 0;
        std::vector<float> tri;
        ok = mesh(nullptr, 0, &nt) == TSDF_OK;
        if (ok) {
            tri.resize(9 * nt);
            ok = mesh(tri.data(), nt, &nt) == TSDF_OK;
        }
        if (!ok) ROS_ERROR("tsdf mesh: %s", tsdf_last_error(tc ? tc : ctx_));
        tsdf_destroy(tc);
        if (!ok) return false;
        const std::string mtmp = mesh_path_ + ".tmp";
        FILE* m = std::fopen(mtmp.c_str(), "wb");  // binary PLY triangle soup
        if (!m) return false;
        std::fprintf(m,
                     "ply\nformat binary_little_endian 1.0\nelement vertex %llu\n"
                     "property float x\nproperty float y\nproperty float z\n"
                     "element face %llu\nproperty list uchar int vertex_indices\nend_header\n",
                     (unsigned long long)(3 * nt), (unsigned long long)nt);
        std::fwrite(tri.data(), 4, 9 * nt, m);
        for (uint64_t t = 0; t < nt; t++) {
            const unsigned char three = 3;
            const int32_t v[3] = {(int32_t)(3 * t), (int32_t)(3 * t + 1), (int32_t)(3 * t + 2)};
            std::fwrite(&three, 1, 1, m);
            std::fwrite(v, 4, 3, m);
        }
        ok = std::fclose(m) == 0 && std::rename(mtmp.c_str(), mesh_path_.c_str()) == 0;
        if (ok) ROS_INFO("saved %llu triangles to %s", (unsigned long long)nt, mesh_path_.c_str());
        return ok;
    }

    tsdf_ctx* ctx_ = nullptr;            // ctxs_[0]: errors, metrics
    tsdf_params params_{};               // the contexts' parameters (the host-merged mesh's context)
    int save_every_ = 999;               // ~save_every_n_clouds (0: only at shutdown / ~save_map)
    uint64_t clouds_ = 0;
    std::vector<tsdf_ctx*> ctxs_;        // one per GPU (sector k of num_gpus)
    int32_t mesh_table_ = TSDF_MC_LORENSEN;
    tsdf_map::MapCore* core_ = nullptr;
    ros::Subscriber sub_cloud_, sub_pose_, sub_path_;
    ros::ServiceServer srv_save_;
    std::string map_path_, mesh_path_;
};

}  // namespace

int main(int argc, char** argv) {
    ros::init(argc, argv, "tsdf_map_node");
    ros::NodeHandle nh, pnh("~");
    TsdfMapNode node(nh, pnh);
    ros::spin();  // single-threaded: the contexts are used by this one thread (include/tsdf_hip.h)
    return 0;
}
